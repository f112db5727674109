// Restart-on-change runner for the dev loop (what `nodemon index.js` does in the reference's
// quickstart, /root/reference/examples/quickstart/package.json:7), with no npm dependencies so
// the offline image needs no `npm install`.
//
//   node watch.js index.js        (npm run dev)
//
// Watches the app directory (devspace sync writes files with an atomic rename, which
// fs.watch reports as a 'rename' event on the directory), stops the running server, waits
// for it to exit so the port is free, and starts it again. Edits that land while a restart is
// in progress coalesce into one more restart.
const {spawn} = require('child_process');
const fs = require('fs');
const path = require('path');

const script = process.argv[2] || 'index.js';
const dir = path.dirname(path.resolve(script));
const ignored = /(^|\/)(node_modules|\.git|\.devspace)(\/|$)|\.sw.$|~$/;
let child = null;
let pending = false;
let restarting = false;
let gen = 0;

function start() {
  gen++;
  child = spawn(process.execPath, [script], {stdio: 'inherit'});
  console.log('[watch] started gen=' + gen + ' pid=' + child.pid);
  child.on('exit', () => {
    child = null;
    if (restarting) {
      restarting = false;
      start();
      if (pending) schedule();
    }
  });
}

function schedule() {
  pending = false;
  if (restarting) {
    pending = true;
    return;
  }
  if (!child) {
    start();
    return;
  }
  restarting = true;
  child.kill('SIGTERM');
}

fs.watch(dir, {persistent: true}, (event, name) => {
  if (!name || ignored.test(name) || !/\.(js|json)$/.test(name)) return;
  schedule();
});
for (const sig of ['SIGINT', 'SIGTERM']) {
  process.on(sig, () => {
    restarting = false;
    if (child) child.kill(sig);
    process.exit(0);
  });
}
start();
