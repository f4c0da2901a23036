'use strict';
// GPU: the multi-GPU group sort from Node (RadixSortGroup over rs_group_*).  RCCL at world size 1
// and 3 virtual ranks on device 0 over the peer-copy transport; every rank's result is read back
// through the WebGPU-shaped copy path and the rank-ordered concatenation is compared with the
// CPU: keys with Uint32Array.sort((a, b) => a - b) (example/tests.ts:86), values with the stable
// order of the global input index (stricter than keys[values[i]] == keys'[i], tests.ts:94).
const assert = require('assert');
const rs = require('..');

function rng(seed) {
  let s = BigInt(seed) * 0x9E3779B97F4A7C15n & 0xFFFFFFFFFFFFFFFFn;
  return () => {
    s = (s + 0x9E3779B97F4A7C15n) & 0xFFFFFFFFFFFFFFFFn;
    let z = s;
    z = ((z ^ (z >> 30n)) * 0xBF58476D1CE4E5B9n) & 0xFFFFFFFFFFFFFFFFn;
    z = ((z ^ (z >> 27n)) * 0x94D049BB133111EBn) & 0xFFFFFFFFFFFFFFFFn;
    return Number((z ^ (z >> 31n)) & 0xFFFFFFFFn);
  };
}

function upload(device, arr) {
  const b = device.createBuffer({ size: arr.byteLength, usage: rs.GPUBufferUsage.STORAGE | rs.GPUBufferUsage.COPY_DST });
  device.queue.writeBuffer(b, 0, arr);
  return b;
}

async function readBack(device, src, count) {
  const dst = device.createBuffer({ size: Math.max(4, count * 4), usage: rs.GPUBufferUsage.MAP_READ | rs.GPUBufferUsage.COPY_DST });
  const enc = device.createCommandEncoder();
  if (count) enc.copyBufferToBuffer(src, 0, dst, 0, count * 4);
  device.queue.submit([enc.finish()]);
  await dst.mapAsync(rs.GPUMapMode.READ);
  return new Uint32Array(dst.getMappedRange().slice(0, count * 4));
}

async function run(devices, counts, transport, hasValues, keyFn) {
  const group = new rs.RadixSortGroup({ devices, capacity: Math.max(...counts), hasValues, transport, rounds: 3 });
  const all = [];
  const slices = counts.map((n, r) => {
    const dev = group.devices[r];
    const k = new Uint32Array(n);
    const v = new Uint32Array(n);
    for (let i = 0; i < n; ++i) { k[i] = keyFn(); v[i] = all.length; all.push(k[i]); }
    return { keys: upload(dev, k), values: hasValues ? upload(dev, v) : undefined, count: n };
  });
  group.sort(slices);
  group.synchronize();
  const gotK = [];
  const gotV = [];
  for (let r = 0; r < group.world; ++r) {
    const res = group.result(r);
    const dev = group.devices[r];
    for (const x of await readBack(dev, res.keys, res.count)) gotK.push(x);
    if (hasValues) for (const x of await readBack(dev, res.values, res.count)) gotV.push(x);
  }
  const keys = Uint32Array.from(all);
  const expK = Uint32Array.from(keys).sort((a, b) => a - b);
  assert.strictEqual(gotK.length, all.length);
  for (let i = 0; i < expK.length; ++i) assert.strictEqual(gotK[i], expK[i], `key ${i}`);
  if (hasValues) {
    const idx = Array.from(keys.keys()).sort((a, b) => keys[a] - keys[b]);   // stable (V8 TimSort)
    for (let i = 0; i < idx.length; ++i) assert.strictEqual(gotV[i], idx[i], `value ${i}`);
  }
  for (const s of slices) { s.keys.destroy(); if (s.values) s.values.destroy(); }
  group.destroy();
}

(async () => {
  const r = rng(7);
  await run([0], [200000], 'rccl', true, r);
  await run([0], [70000], 'rccl', false, r);
  await run([0, 0, 0], [120000, 3, 50000], 'copy', true, r);
  await run([0, 0, 0], [40000, 40000, 0], 'copy', false, () => (r() & 0xFF) << 24);   // heavy duplicates
  console.log('node group checks ok');
})().catch((e) => { console.error(e); process.exit(1); });
