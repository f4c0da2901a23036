// Evaluates the reference test's own expected-value expressions in Node (fixture generation
// only; see gen_golden.py).  Restated, not copied:
//   sort:  keys.slice(0, count).sort((a, b) => a - b)      (example/tests.ts:86)
//   scan:  exclusive running sum, as prefixSumCpu          (example/tests.ts:288-296)
// usage: node node_expected.js sort|scan <in.bin> <count> <out.bin>
'use strict';
const fs = require('fs');
const [mode, inPath, countStr, outPath] = process.argv.slice(2);
const buf = fs.readFileSync(inPath);
const data = new Uint32Array(buf.buffer, buf.byteOffset, buf.byteLength / 4);
const count = Number(countStr);
let out;
if (mode === 'sort') {
  out = data.slice(0, count).sort((a, b) => a - b);
} else if (mode === 'scan') {
  out = new Uint32Array(count);
  let sum = 0;
  for (let i = 0; i < count; i += 1) { out[i] = sum; sum = (sum + data[i]) >>> 0; }
} else {
  throw new Error('mode must be sort|scan');
}
fs.writeFileSync(outPath, Buffer.from(out.buffer, out.byteOffset, out.byteLength));
