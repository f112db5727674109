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
//
// Every restart is a fresh process, as with nodemon, but not a cold one: standby node
// processes are kept booted (V8 + core modules initialised, nothing of the app loaded). A
// restart hands the script to a booted standby, which loads it then — from disk, after the
// edit — as its main module (`require.main === module` holds), and a replacement boots in the
// background. That takes node's start-up (tens of ms) out of every edit -> response.
//
// The pool adapts to the edit rate: it starts at WATCH_STANDBY (default 4) standbys, grows by
// one (up to WATCH_STANDBY_MAX, default 8) whenever a restart finds none of them booted —
// back-to-back saves (format-on-save, generated files, a script editing in a loop) come faster
// than node boots — and gives one back after 30 s (WATCH_STANDBY_SHRINK_MS) without such a miss. A standby that finished
// booting a while ago also starts the app faster than a just-booted one (~10 ms on the MI355X
// box, profiles/r3_qs_standby_probe.txt). WATCH_STANDBY=0 gives plain cold restarts.
const {spawn} = require('child_process');
const fs = require('fs');
const path = require('path');

const script = path.resolve(process.argv[2] || 'index.js');
const dir = path.dirname(script);
const ignored = /(^|\/)(node_modules|\.git|\.devspace)(\/|$)|\.sw.$|~$/;
const minStandby = Math.max(0, parseInt(process.env.WATCH_STANDBY || '4', 10) || 0);
const maxStandby = minStandby && Math.max(minStandby, parseInt(process.env.WATCH_STANDBY_MAX || '8', 10) || 0);
const shrinkMs = parseInt(process.env.WATCH_STANDBY_SHRINK_MS || '30000', 10) || 30000;
let nStandby = minStandby;
let lastMiss = 0;  // time of the last restart that found no booted standby
// The standby's whole program: load the core modules a server needs (node loads them lazily,
// and they are shared, stateless code: nothing of the app), wait for the go signal, close its
// pipe to the watcher (the app must not see it) and run the script as the main module.
// `cluster` and `child_process` are in the list because net's listen() loads them on first
// use. The boot also warms the runtime paths every server takes once: it compiles a module
// from a string (the CommonJS wrapper/compiler), and it serves one HTTP request to itself on an
// ephemeral loopback port, then closes that server (libuv's TCP setup, net's listen path, the
// HTTP parser and response writer). Measured with node 12, the first listen() of a booted
// process took 6-9 ms to reach its callback and 0.4 ms after a listen warm-up
// (scripts/node_boot_probe.py); the first request to the new server took 7.7 ms after the
// listen warm-up and 1.8 ms after the request warm-up (CPU container). Nothing of the app runs
// before the go signal.
const PRELOAD = ['http', 'https', 'net', 'url', 'querystring', 'stream', 'events', 'util', 'crypto',
                 'zlib', 'os', 'fs', 'path', 'buffer', 'string_decoder', 'timers', 'dns', 'cluster',
                 'child_process'];
const WARM = "const M = require('module'); const w = new M('/.watch-warm.js'); " +
    "w.filename = '/.watch-warm.js'; w.paths = []; w._compile('module.exports = 0;', '/.watch-warm.js'); " +
    "const http = require('http'); setTimeout(ready, 3000).unref(); " +
    "const ws = warm = http.createServer((q, r) => { r.writeHead(200, {'Content-Type': 'text/plain'}); r.end('w'); }); " +
    "const done = () => { try { ws.close(() => ready()); } catch (e) { ready(); } }; " +
    "ws.on('error', ready); " +
    "ws.listen(0, '127.0.0.1', () => { try { " +
    "const req = http.get({host: '127.0.0.1', port: ws.address().port, path: '/', agent: false}, (res) => { " +
    "res.resume(); res.on('end', done); res.on('error', done); }); req.on('error', done); " +
    "} catch (e) { done(); } });\n";
// The hand-off goes by a signal, not a message: the standby talks to the watcher on a plain
// pipe (fd 3: 'b' once its SIGUSR2 handler is installed, 'r' once warmed up) and starts the app
// on SIGUSR2, after closing fd 3. Node's IPC channel cost more: on the MI355X box the old
// server's kill -> new server listening went from 4.31 to 3.55 ms and the loop's p90 dropped
// 0.3-0.5 ms (profiles/r3_watch_signal_handoff_ab.txt), most of the gap in
// process.disconnect(). The app sees no trace of either: no process.send, no fd 3, no SIGUSR2
// listener. The watcher signals only after 'b' (SIGUSR2's default action ends a
// process that has no handler yet), and a standby exits when the pipe's other end closes (the
// watcher died), as it did with the IPC channel. A standby can be handed the script before its
// warm-up finished (a restart that found none booted): the go then ends the warm-up (its server
// closes, `ready` turns into a no-op) and the app runs.
const BOOT = "const ctl = new (require('net').Socket)({fd: 3, readable: true, writable: true});\n" +
    "ctl.on('error', () => {}); ctl.on('end', () => process.exit(0)); ctl.resume();\n" +
    "let sent = false, warm = null;\n" +
    "process.once('SIGUSR2', () => { " +
    "sent = true; if (warm) { try { warm.close(); } catch (e) {} warm = null; } " +
    `ctl.removeAllListeners('end'); ctl.destroy(); process.argv[1] = ${JSON.stringify(script)}; ` +
    "require('module').runMain(); });\n" +
    "ctl.write('b');\n" +
    `for (const m of ${JSON.stringify(PRELOAD)}) { try { require(m); } catch (e) {} }\n` +
    "function ready() { if (!sent) { sent = true; ctl.write('r'); } }\n" +
    `try { ${WARM} } catch (e) { ready(); }\n`;
let child = null;
let standbys = [];  // booting or booted, oldest first
let pending = false;
let restarting = false;
let gen = 0;

function bootStandbys() {
  while (standbys.length < nStandby) {
    const s = spawn(process.execPath, ['-e', BOOT], {stdio: ['inherit', 'inherit', 'inherit', 'pipe']});
    s.armed = false;  // its SIGUSR2 handler is installed
    s.ready = false;  // warmed up
    s.onArmed = null;
    s.stdio[3].on('error', () => {});
    s.stdio[3].on('data', (d) => {
      d = String(d);
      if (d.includes('b')) s.armed = true;
      if (d.includes('r')) s.ready = true;
      if (s.armed && s.onArmed) {
        const go = s.onArmed;
        s.onArmed = null;
        go();
      }
    });
    s.on('exit', () => {
      standbys = standbys.filter((x) => x !== s);
    });
    standbys.push(s);
  }
}

function resize(ready) {
  const now = Date.now();
  if (!ready && nStandby > 0) {
    lastMiss = now;
    nStandby = Math.min(maxStandby, nStandby + 1);
  } else if (nStandby > minStandby && now - lastMiss > shrinkMs) {
    lastMiss = now;  // one step down per quiet period (WATCH_STANDBY_SHRINK_MS, 30 s)
    nStandby--;
    // drop standbys still booting first, then the youngest booted ones
    let extra = standbys.length - nStandby;
    for (let k = standbys.length - 1; k >= 0 && extra > 0; k--) {
      if (!standbys[k].ready) {
        standbys.splice(k, 1)[0].kill('SIGKILL');
        extra--;
      }
    }
    for (; extra > 0; extra--) standbys.pop().kill('SIGKILL');
  }
}

function start() {
  gen++;
  // a booted standby if there is one, else the one that started booting first
  if (gen > 1) resize(standbys.some((x) => x.ready));  // the first start has no pool yet: not a miss
  const i = standbys.findIndex((x) => x.ready);  // after resize: a shrink may drop pool members
  const s = standbys.splice(i >= 0 ? i : 0, 1)[0];
  if (s) {
    child = s;
    const go = () => s.kill('SIGUSR2');
    if (s.armed) go();
    else s.onArmed = go;
  } else {
    child = spawn(process.execPath, [script], {stdio: 'inherit'});
  }
  console.log('[watch] started gen=' + gen + ' pid=' + child.pid + (s ? ' (standby' + (s.ready ? ')' : ', booting)') : ''));
  const me = child;
  me.on('exit', () => {
    if (child !== me) return;
    child = null;
    if (restarting) {
      restarting = false;
      start();
      if (pending) schedule();
    }
  });
  setImmediate(bootStandbys);
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
    for (const x of standbys) x.kill('SIGKILL');
    if (child) child.kill(sig);
    process.exit(0);
  });
}
start();
