// A tiny HTTP service for developing against a local minikube node (no npm dependencies).
const http = require('http');
const port = Number(process.env.PORT || 3000);
const started = new Date().toISOString();
http.createServer((req, res) => {
  res.writeHead(200, {'Content-Type': 'application/json'});
  res.end(JSON.stringify({hello: 'minikube', pod: process.env.HOSTNAME || 'local', started}) + '\n');
}).listen(port, () => console.log(`listening on ${port}`));
