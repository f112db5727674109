// Minimal HTTP service (no npm dependencies, so the offline local cluster can run it).
const http = require('http');
const port = process.env.PORT || 3000;
http.createServer((req, res) => {
  res.writeHead(200, {'Content-Type': 'text/plain'});
  res.end('Hello from ' + (process.env.HOSTNAME || 'devspace') + '\n');
}).listen(port, () => console.log('Example app listening on port ' + port + '!'));
