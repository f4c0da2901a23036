'use strict';
// CPU-only checks of the Node façade: the addon loads, exports the reference's classes, and
// validates options exactly where the reference throws (no GPU needed: validation happens
// before any device call).
const assert = require('assert');
const rs = require('..');

for (const name of ['RadixSortKernel', 'RadixSortBufferKernel', 'RadixSortTextureKernel', 'PrefixSumKernel', 'gpu',
  'GPUBufferUsage', 'GPUMapMode']) {
  assert.ok(rs[name], `missing export ${name}`);
}
assert.strictEqual(typeof rs.addon.planCreate, 'function');
assert.strictEqual(rs.addon.FLAG_INTERLEAVED, 0x10);
assert.strictEqual(rs.addon.version(), 1);

const fakeKeys = { ptr: 4096n };
// PrefixSumKernel.ts:33-35: non power-of-two workgroups throw
assert.throws(() => new rs.RadixSortKernel({ keys: fakeKeys, count: 10, workgroup_size: { x: 3, y: 3 } }),
  /power of two/);
assert.throws(() => new rs.RadixSortBufferKernel({ data: { keys: fakeKeys }, count: 10, workgroupSize: { x: 6, y: 1 } }),
  /power of two/);
assert.throws(() => new rs.PrefixSumKernel({ data: fakeKeys, count: 10, workgroupSize: { x: 12, y: 1 } }),
  /power of two/);
// README.md:97: bit_count must be a multiple of 4
assert.throws(() => new rs.RadixSortKernel({ keys: fakeKeys, count: 10, bit_count: 6 }), /bit_count/);
assert.throws(() => new rs.RadixSortKernel({ data: { keys: fakeKeys }, count: 10, bitCount: 36 }), /bit_count/);
assert.throws(() => new rs.RadixSortKernel({ count: 10 }), /keys buffer is required/);
assert.throws(() => new rs.RadixSortKernel({ keys: fakeKeys }), /count is required/);
assert.throws(() => new rs.RadixSortTextureKernel({ count: 10 }), /texture is required/);
assert.throws(() => new rs.RadixSortTextureKernel({ data: { texture: { ptr: 4096n, format: 'r32uint' } }, count: 10 }),
  /rg32uint/);
console.log('node api checks ok');
