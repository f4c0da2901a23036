'use strict';
// GPU: the reference's own test flow (example/tests.ts:9-107), seeded: create buffers,
// construct the kernel, dispatch into a compute pass, copy back, submit, mapAsync, compare
// against keys.slice(0, count).sort((a, b) => a - b) and keysResult[i] == keys[values[i]];
// additionally checks stability (values = iota stay increasing within equal keys) and the
// prefix sum against prefixSumCpu (example/tests.ts:288-296).
const assert = require('assert');
const { gpu, RadixSortKernel, RadixSortBufferKernel, RadixSortTextureKernel, PrefixSumKernel, GPUBufferUsage, GPUMapMode } = require('..');

function mulberry32(a) {
  return function next() {
    a |= 0; a = (a + 0x6D2B79F5) | 0;
    let t = Math.imul(a ^ (a >>> 15), 1 | a);
    t = (t + Math.imul(t ^ (t >>> 7), 61 | t)) ^ t;
    return ((t ^ (t >>> 14)) >>> 0) / 4294967296;
  };
}

function createBuffers(device, data) {       // example/tests.ts:227-244
  const dataBuffer = device.createBuffer({ size: data.length * 4, usage: GPUBufferUsage.STORAGE | GPUBufferUsage.COPY_SRC, mappedAtCreation: true });
  new Uint32Array(dataBuffer.getMappedRange()).set(data);
  dataBuffer.unmap();
  const dataBufferMapped = device.createBuffer({ size: data.length * 4, usage: GPUBufferUsage.MAP_READ | GPUBufferUsage.COPY_DST });
  return [dataBuffer, dataBufferMapped];
}

async function testRadixSort(device, keysAndValues, rand) {
  let cases = 0;
  for (const [wx, wy] of [[16, 16], [8, 4], [32, 32], [2, 2]]) {
    for (let exp = 2; exp < 7; exp += 1) {
      const elementCount = Math.floor(10 ** exp * (rand() * 0.1 + 0.9));
      const subElementCount = Math.floor(elementCount * rand() + 1);
      const keys = new Uint32Array(elementCount).map(() => Math.ceil(rand() * (2 ** 32 - 1)) % (exp === 3 ? 97 : 2 ** 32));
      const values = new Uint32Array(elementCount).map((_, i) => i);
      const checkOrder = rand() > 0.5;
      const localShuffle = rand() > 0.5;
      const avoidBankConflicts = rand() > 0.5;
      const [keysBuffer, keysBufferMapped] = createBuffers(device, keys);
      const [valuesBuffer, valuesBufferMapped] = createBuffers(device, values);
      const Kernel = rand() > 0.5 ? RadixSortKernel : RadixSortBufferKernel;
      const kernel = new Kernel({
        device, data: { keys: keysBuffer, values: keysAndValues ? valuesBuffer : undefined },
        count: subElementCount, bitCount: 32, workgroupSize: { x: wx, y: wy },
        checkOrder, localShuffle, avoidBankConflicts,
      });
      const encoder = device.createCommandEncoder();
      const pass = encoder.beginComputePass();
      kernel.dispatch(pass);
      pass.end();
      encoder.copyBufferToBuffer(kernel.buffers.keys, 0, keysBufferMapped, 0, elementCount * 4);
      if (keysAndValues) encoder.copyBufferToBuffer(kernel.buffers.values, 0, valuesBufferMapped, 0, elementCount * 4);
      device.queue.submit([encoder.finish()]);
      await keysBufferMapped.mapAsync(GPUMapMode.READ);
      const keysResult = new Uint32Array(keysBufferMapped.getMappedRange().slice());
      keysBufferMapped.unmap();
      const expected = keys.slice(0, subElementCount).sort((a, b) => a - b);
      assert.ok(expected.every((v, i) => v === keysResult[i]), `keys mismatch n=${elementCount} count=${subElementCount}`);
      for (let i = subElementCount; i < elementCount; i += 1) assert.strictEqual(keysResult[i], keys[i]);
      if (keysAndValues) {
        await valuesBufferMapped.mapAsync(GPUMapMode.READ);
        const valuesResult = new Uint32Array(valuesBufferMapped.getMappedRange().slice());
        valuesBufferMapped.unmap();
        for (let i = 0; i < subElementCount; i += 1) {
          assert.strictEqual(keysResult[i], keys[valuesResult[i]]);
          if (i && keysResult[i] === keysResult[i - 1]) assert.ok(valuesResult[i] > valuesResult[i - 1], 'stability');
        }
      }
      kernel.destroy();
      for (const b of [keysBuffer, valuesBuffer]) b.destroy();
      cases += 1;
    }
  }
  return cases;
}

async function testPrefixSum(device, rand) {
  for (const n of [1, 7, 512, 1025, 100003]) {
    const data = new Uint32Array(n).map(() => Math.floor(rand() * 8));
    const [buf, mapped] = createBuffers(device, data);
    const k = new PrefixSumKernel({ device, data: buf, count: n, workgroupSize: { x: 16, y: 16 } });
    const encoder = device.createCommandEncoder();
    const pass = encoder.beginComputePass();
    k.dispatch(pass);
    pass.end();
    encoder.copyBufferToBuffer(buf, 0, mapped, 0, n * 4);
    device.queue.submit([encoder.finish()]);
    await mapped.mapAsync(GPUMapMode.READ);
    const out = new Uint32Array(mapped.getMappedRange().slice());
    let sum = 0;
    for (let i = 0; i < n; i += 1) { assert.strictEqual(out[i], sum >>> 0); sum += data[i]; }
    k.destroy();
    buf.destroy();
  }
}

// RadixSortTextureKernel (RadixSortTextureKernel.ts:15-35): an rg32uint (key, value) texture,
// written with queue.writeTexture, sorted in place, read back with copyTextureToBuffer.
async function testTextureSort(device, rand) {
  let cases = 0;
  for (const [w, h] of [[16, 4], [256, 40], [1000, 123], [2048, 512]]) {
    const n = w * h;
    const count = rand() > 0.5 ? n : Math.floor(n * rand()) + 1;
    const texels = new Uint32Array(2 * n);
    for (let i = 0; i < n; i += 1) {
      texels[2 * i] = Math.floor(rand() * 2 ** 32) % (cases === 1 ? 61 : 2 ** 32);
      texels[2 * i + 1] = i;
    }
    const texture = device.createTexture({ size: { width: w, height: h }, format: 'rg32uint' });
    device.queue.writeTexture({ texture }, texels, { bytesPerRow: w * 8 }, { width: w, height: h });
    const kernel = new RadixSortTextureKernel({ device, data: { texture }, count, bitCount: 32,
      checkOrder: rand() > 0.5 });
    const out = device.createBuffer({ size: n * 8, usage: GPUBufferUsage.MAP_READ | GPUBufferUsage.COPY_DST });
    const encoder = device.createCommandEncoder();
    const pass = encoder.beginComputePass();
    kernel.dispatch(pass);
    pass.end();
    encoder.copyTextureToBuffer({ texture }, { buffer: out, bytesPerRow: w * 8 }, { width: w, height: h });
    device.queue.submit([encoder.finish()]);
    await out.mapAsync(GPUMapMode.READ);
    const r = new Uint32Array(out.getMappedRange().slice());
    const idx = Array.from({ length: count }, (_, i) => i)
      .sort((a, b) => (texels[2 * a] - texels[2 * b]) || (a - b));   // stable by key
    for (let i = 0; i < count; i += 1) {
      assert.strictEqual(r[2 * i], texels[2 * idx[i]], `texture key ${w}x${h} @${i}`);
      assert.strictEqual(r[2 * i + 1], idx[i], `texture value ${w}x${h} @${i}`);
    }
    for (let i = 2 * count; i < 2 * n; i += 1) assert.strictEqual(r[i], texels[i]);
    kernel.destroy();
    texture.destroy();
    cases += 1;
  }
  return cases;
}

// Skewed f32 keys on the hybrid path (>= 12M: half of the keys in [0, 1) share 128 16-bit buckets
// of ~n/256 records): the over-full buckets are split, not sent to the LSD fallback.
async function testSkewedFloatKeys(device, rand) {
  const n = 12 * 1024 * 1024 + 77;
  const f = new Float32Array(n);
  for (let i = 0; i < n; i += 1) f[i] = Math.floor(rand() * 2 ** 24) * 2 ** -24;
  const keys = new Uint32Array(f.buffer);
  const values = new Uint32Array(n).map((_, i) => i);
  const [keysBuffer, keysBufferMapped] = createBuffers(device, keys);
  const [valuesBuffer, valuesBufferMapped] = createBuffers(device, values);
  const kernel = new RadixSortKernel({ device, data: { keys: keysBuffer, values: valuesBuffer }, count: n, bitCount: 32 });
  const encoder = device.createCommandEncoder();
  const pass = encoder.beginComputePass();
  kernel.dispatch(pass);
  pass.end();
  encoder.copyBufferToBuffer(kernel.buffers.keys, 0, keysBufferMapped, 0, n * 4);
  encoder.copyBufferToBuffer(kernel.buffers.values, 0, valuesBufferMapped, 0, n * 4);
  device.queue.submit([encoder.finish()]);
  await keysBufferMapped.mapAsync(GPUMapMode.READ);
  await valuesBufferMapped.mapAsync(GPUMapMode.READ);
  const kr = new Uint32Array(keysBufferMapped.getMappedRange().slice());
  const vr = new Uint32Array(valuesBufferMapped.getMappedRange().slice());
  keysBufferMapped.unmap();
  valuesBufferMapped.unmap();
  assert.strictEqual(kernel.lastPath(), 'hybrid');
  assert.ok(kernel.lastSplit() >= 2, `split levels ${kernel.lastSplit()}`);
  const expected = keys.slice().sort();
  for (let i = 0; i < n; i += 1) {
    assert.strictEqual(kr[i], expected[i], `f32 key @${i}`);
    assert.strictEqual(kr[i], keys[vr[i]], `f32 value @${i}`);
    if (i && kr[i] === kr[i - 1]) assert.ok(vr[i] > vr[i - 1], 'stability');
  }
  kernel.destroy();
  for (const b of [keysBuffer, valuesBuffer]) b.destroy();
}

// Nearly-sorted keys with checkOrder (>= 12M): the presorted path sorts them, and lastPath() names
// it "presorted" (the addon's path-name table covers every RS_PATH_* value).
async function testPresortedPath(device, rand) {
  const n = 12 * 1024 * 1024 + 5;
  const keys = new Uint32Array(n);
  for (let i = 0; i < n; i += 1) keys[i] = i * 3;
  for (let s = 0; s < 2000; s += 1) {   // transpositions of neighbours a few places apart
    const i = Math.floor(rand() * (n - 8));
    const j = i + 1 + Math.floor(rand() * 6);
    const t = keys[i]; keys[i] = keys[j]; keys[j] = t;
  }
  const [keysBuffer, keysBufferMapped] = createBuffers(device, keys);
  const kernel = new RadixSortKernel({ device, data: { keys: keysBuffer }, count: n, bitCount: 32, checkOrder: true });
  const encoder = device.createCommandEncoder();
  const pass = encoder.beginComputePass();
  kernel.dispatch(pass);
  pass.end();
  encoder.copyBufferToBuffer(kernel.buffers.keys, 0, keysBufferMapped, 0, n * 4);
  device.queue.submit([encoder.finish()]);
  await keysBufferMapped.mapAsync(GPUMapMode.READ);
  const kr = new Uint32Array(keysBufferMapped.getMappedRange().slice());
  keysBufferMapped.unmap();
  assert.strictEqual(kernel.lastPath(), 'presorted');
  for (let i = 0; i < n; i += 1) assert.strictEqual(kr[i], i * 3, `presorted key @${i}`);
  kernel.destroy();
  keysBuffer.destroy();
}

(async () => {
  const adapter = await gpu.requestAdapter();
  assert.ok(adapter, 'no HIP device');
  const device = await adapter.requestDevice();
  const rand = mulberry32(20250404);
  const a = await testRadixSort(device, false, rand);
  const b = await testRadixSort(device, true, rand);
  const c = await testTextureSort(device, rand);
  await testPrefixSum(device, rand);
  await testSkewedFloatKeys(device, rand);
  await testPresortedPath(device, rand);
  console.log(`node sort checks ok (${a + b} sort cases, ${c} texture cases, prefix sum, skewed f32 hybrid split, presorted path)`);
})().catch((e) => { console.error(e); process.exit(1); });
