# Rebuilt + redeployed on every change (dev.autoReload.paths) instead of syncing.
import http.server
import os

MESSAGE = "Hello from a redeployed pod"


class H(http.server.BaseHTTPRequestHandler):
    def do_GET(self):
        body = (MESSAGE + "\n").encode()
        self.send_response(200)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)


if __name__ == "__main__":
    print(MESSAGE, flush=True)
    http.server.ThreadingHTTPServer(("0.0.0.0", int(os.environ.get("PORT", "8081"))), H).serve_forever()
