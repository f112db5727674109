# Tiny HTTP service built in-cluster by kaniko (no local docker daemon needed).
import http.server
import os


class Hello(http.server.BaseHTTPRequestHandler):
    def do_GET(self):
        body = ("Hello from %s (built with kaniko)\n" % os.environ.get("HOSTNAME", "pod")).encode()
        self.send_response(200)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)


if __name__ == "__main__":
    port = int(os.environ.get("PORT", "8080"))
    print("listening on", port, flush=True)
    http.server.ThreadingHTTPServer(("0.0.0.0", port), Hello).serve_forever()
