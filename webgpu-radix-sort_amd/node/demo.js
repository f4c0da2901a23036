#!/usr/bin/env node
'use strict';
// Command-line counterpart of the reference's demo page (example/index.ts): the same `settings`
// (:4-15), the same data generation for buffers (:44-87) and textures (:89-120), the sort timed
// on the GPU between the compute pass's beginning/end timestamp writes (:125-146, via
// createTimestampQuery, example/tests.ts:247-285), the CPU reference `keys.sort((a, b) => a - b)`
// timed on the first run only (:148-152), and the same report (:155-181) as plain text.
//
//   node demo.js --elementCount=1048576 --sortMode="Keys & Values" --dataType=texture \
//        --consecutiveSorts=10 [--seed=1] [--verify] [--json]
//
// Differences from the page: the generator is a seeded mulberry32 instead of Math.random (runs
// are reproducible), --verify compares the GPU result with the CPU one, --json prints one JSON
// line instead of the text report.
const { gpu, RadixSortBufferKernel, RadixSortTextureKernel, GPUBufferUsage, GPUMapMode } = require('.');

const settings = {
  dataType: 'buffer',          // 'buffer' | 'texture'
  elementCount: 2 ** 20,
  bitCount: 32,
  workgroupSize: 16,
  checkOrder: false,
  localShuffle: false,
  avoidBankConflicts: false,
  sortMode: 'Keys',            // 'Keys' | 'Keys & Values'
  initialSort: 'Random',       // 'Random' | 'Sorted'
  consecutiveSorts: 1,
};
const extra = { seed: 1, verify: false, json: false };

function parseArgs(argv) {
  for (const a of argv) {
    const m = /^--([A-Za-z]+)(?:=(.*))?$/.exec(a);
    if (!m) throw new Error(`bad argument ${a}`);
    const [, key, raw] = m;
    const target = key in settings ? settings : (key in extra ? extra : null);
    if (!target) throw new Error(`unknown setting ${key}`);
    const cur = target[key];
    if (typeof cur === 'boolean') target[key] = raw === undefined || raw === 'true' || raw === '1';
    else if (typeof cur === 'number') target[key] = Number(raw);
    else target[key] = raw;
  }
}

function mulberry32(a) {
  return function next() {
    a |= 0; a = (a + 0x6D2B79F5) | 0;
    let t = Math.imul(a ^ (a >>> 15), 1 | a);
    t = (t + Math.imul(t ^ (t >>> 7), 61 | t)) ^ t;
    return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
  };
}

function createBuffer(device, data) {         // example/tests.ts:227-244 (upload half)
  const buf = device.createBuffer({ size: data.byteLength, usage: GPUBufferUsage.STORAGE | GPUBufferUsage.COPY_SRC, mappedAtCreation: true });
  new Uint32Array(buf.getMappedRange()).set(data);
  buf.unmap();
  return buf;
}

function sortWithBuffers(device, rand) {       // example/index.ts:44-87
  const n = settings.elementCount;
  const keys = new Uint32Array(n);
  const keysRange = 2 ** settings.bitCount;
  if (settings.initialSort === 'Random') for (let i = 0; i < n; i += 1) keys[i] = Math.floor(rand() * keysRange);
  else for (let i = 0; i < n; i += 1) keys[i] = i;
  const keysBuffer = createBuffer(device, keys);
  let valuesBuffer;
  if (settings.sortMode === 'Keys & Values') {
    const values = new Uint32Array(n);
    for (let i = 0; i < n; i += 1) values[i] = Math.floor(rand() * 1000000);
    valuesBuffer = createBuffer(device, values);
  }
  const kernel = new RadixSortBufferKernel({
    device, data: { keys: keysBuffer, values: valuesBuffer }, count: n, bitCount: settings.bitCount,
    workgroupSize: { x: settings.workgroupSize, y: settings.workgroupSize },
    checkOrder: settings.checkOrder, localShuffle: settings.localShuffle,
    avoidBankConflicts: settings.avoidBankConflicts,
  });
  return {
    kernel,
    sort: () => keys.sort((a, b) => a - b),
    result: keysBuffer,
    stride: 1,
    release: () => { keysBuffer.destroy(); if (valuesBuffer) valuesBuffer.destroy(); },
  };
}

function sortWithTextures(device, rand) {      // example/index.ts:89-120
  const n = settings.elementCount;
  const data = new Uint32Array(2 * n);
  const keysRange = 2 ** settings.bitCount;
  for (let i = 0; i < n; i += 1) {
    data[2 * i] = settings.initialSort === 'Random' ? Math.floor(rand() * keysRange) : i;
    data[2 * i + 1] = Math.floor(rand() * 1000000);
  }
  // a square-ish rg32uint texture, as createTexture in example/tests.ts does
  const width = Math.min(n, 8192);
  const height = Math.ceil(n / width);
  const texture = device.createTexture({ size: { width, height }, format: 'rg32uint' });
  const padded = new Uint32Array(2 * width * height);
  padded.set(data);
  device.queue.writeTexture({ texture }, padded, { bytesPerRow: width * 8 }, { width, height });
  const kernel = new RadixSortTextureKernel({
    device, data: { texture }, count: n, bitCount: settings.bitCount,
    workgroupSize: { x: settings.workgroupSize, y: settings.workgroupSize },
    checkOrder: settings.checkOrder, avoidBankConflicts: settings.avoidBankConflicts,
  });
  return {
    kernel,
    sort: () => Uint32Array.from({ length: n }, (_, i) => data[2 * i]).sort((a, b) => a - b),
    result: texture,
    stride: 2,
    release: () => texture.destroy(),
  };
}

async function runSort(device, rand, compareAgainstCpu) {   // example/index.ts:125-154
  const job = settings.dataType === 'buffer' ? sortWithBuffers(device, rand) : sortWithTextures(device, rand);
  const querySet = device.createQuerySet({ type: 'timestamp', count: 2 });
  const queryBuffer = device.createBuffer({ size: 16, usage: GPUBufferUsage.QUERY_RESOLVE | GPUBufferUsage.COPY_SRC });
  const queryResult = device.createBuffer({ size: 16, usage: GPUBufferUsage.MAP_READ | GPUBufferUsage.COPY_DST });
  const encoder = device.createCommandEncoder();
  const pass = encoder.beginComputePass({ timestampWrites: { querySet, beginningOfPassWriteIndex: 0, endOfPassWriteIndex: 1 } });
  job.kernel.dispatch(pass);
  pass.end();
  encoder.resolveQuerySet(querySet, 0, 2, queryBuffer, 0);
  encoder.copyBufferToBuffer(queryBuffer, 0, queryResult, 0, 16);
  device.queue.submit([encoder.finish()]);
  await queryResult.mapAsync(GPUMapMode.READ);
  const ts = new BigUint64Array(queryResult.getMappedRange().slice());
  queryResult.unmap();
  const times = { cpu: 0, gpu: Number(ts[1] - ts[0]) / 1e6, verified: null };
  if (compareAgainstCpu) {
    const start = process.hrtime.bigint();
    const sorted = job.sort();
    times.cpu = Number(process.hrtime.bigint() - start) / 1e6;
    if (extra.verify) {
      const n = settings.elementCount;
      const out = device.createBuffer({ size: n * 4 * job.stride, usage: GPUBufferUsage.MAP_READ | GPUBufferUsage.COPY_DST });
      const enc = device.createCommandEncoder();
      enc.copyBufferToBuffer(job.result, 0, out, 0, n * 4 * job.stride);
      device.queue.submit([enc.finish()]);
      await out.mapAsync(GPUMapMode.READ);
      const r = new Uint32Array(out.getMappedRange());
      let ok = true;
      for (let i = 0; i < n && ok; i += 1) ok = r[i * job.stride] === sorted[i];
      times.verified = ok;
    }
  }
  job.kernel.destroy();
  job.release();
  querySet.destroy();
  queryBuffer.destroy();
  return times;
}

function pretty(n) { return n.toString().replace(/\B(?=(\d{3})+(?!\d))/g, ','); }

async function main() {
  parseArgs(process.argv.slice(2));
  const adapter = await gpu.requestAdapter();
  if (!adapter) throw new Error('Could not create a HIP device');
  const device = await adapter.requestDevice();
  const rand = mulberry32(extra.seed);
  let cpuTime = 0;
  let gpuTime = 0;
  let verified = null;
  for (let i = 0; i < settings.consecutiveSorts; i += 1) {
    const t = await runSort(device, rand, i === 0);
    cpuTime += t.cpu;
    gpuTime += t.gpu;
    if (i === 0) verified = t.verified;
  }
  const gpuAverage = gpuTime / settings.consecutiveSorts;
  const speedup = cpuTime / gpuAverage;
  if (extra.json) {
    console.log(JSON.stringify({ settings, seed: extra.seed, cpu_ms: cpuTime, gpu_avg_ms: gpuAverage, speedup, verified,
      gpu_mkeys_per_s: settings.elementCount / gpuAverage / 1e3 }));
    return;
  }
  console.log(`[1] Sorting ${pretty(settings.elementCount)} ${settings.sortMode.toLowerCase()} of ${settings.bitCount} bits`);
  console.log(`Initial sort: ${settings.initialSort}, Workgroup size: ${settings.workgroupSize}x${settings.workgroupSize}, Data type: ${settings.dataType}`);
  console.log(`Optimizations: (${settings.checkOrder}, ${settings.localShuffle}, ${settings.avoidBankConflicts})`);
  console.log(`> CPU Reference: ${cpuTime.toFixed(2)}ms, GPU Average (${settings.consecutiveSorts} sorts): ${gpuAverage.toFixed(3)}ms, Speedup: x${speedup.toFixed(2)}`
    + (verified === null ? '' : `, GPU result ${verified ? 'matches' : 'DIFFERS FROM'} CPU`));
  if (verified === false) process.exitCode = 1;
}

main().catch((e) => { console.error(e); process.exit(1); });
