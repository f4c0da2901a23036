// The reference's CPU sort path, restated for the CPU baseline (bench.py cpu_baseline leg):
//   keys.sort((a, b) => a - b) on a Uint32Array   (example/index.ts:85,147-151; the same
//   expression is the reference test oracle, example/tests.ts:86)
// timed with performance.now() like example/index.ts:147-151.  Single-threaded V8.
// usage: node cpu_sort_ref.js <keys.bin> -> prints one JSON line
'use strict';
const fs = require('fs');
const os = require('os');
const { performance } = require('perf_hooks');

const buf = fs.readFileSync(process.argv[2]);
const keys = new Uint32Array(buf.buffer, buf.byteOffset, buf.byteLength / 4).slice();
const start = performance.now();
keys.sort((a, b) => a - b);
const ms = performance.now() - start;
let ok = true;
for (let i = 1; i < keys.length; i += 1) if (keys[i - 1] > keys[i]) { ok = false; break; }
console.log(JSON.stringify({
  n: keys.length, ms, sorted: ok, node: process.version,
  cpu_model: (os.cpus()[0] || {}).model, cpus: os.cpus().length,
}));
