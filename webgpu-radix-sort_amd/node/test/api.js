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
assert.strictEqual(rs.addon.version(), 6);
for (const f of ['planCheck', 'scanPlanRunIndirect', 'scanPlanDispatchChain']) {
  assert.strictEqual(typeof rs.addon[f], 'function', f);
}
// argument conversion never truncates silently: negative / over-wide BigInts, fractional or
// negative Numbers and option values above 2^32 - 1 are TypeErrors (before any device call)
assert.throws(() => rs.addon.malloc(0, -1n), TypeError);
assert.throws(() => rs.addon.malloc(0, 2n ** 64n), TypeError);
assert.throws(() => rs.addon.malloc(0, 1.5), TypeError);
assert.throws(() => rs.addon.free(-4096), TypeError);
assert.throws(() => rs.addon.planCreate({ count: 10, bitCount: 2 ** 32 + 8 }), TypeError);
assert.throws(() => rs.addon.planSort(undefined, 1n, null, null), TypeError);

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
// multi-GPU group: options validated before any device call (rs_group_create)
assert.strictEqual(typeof rs.RadixSortGroup, 'function');
for (const f of ['groupCreate', 'groupSort', 'groupResult', 'groupSynchronize', 'groupDestroy']) {
  assert.strictEqual(typeof rs.addon[f], 'function', f);
}
assert.throws(() => new rs.RadixSortGroup({ devices: [], capacity: 10 }), TypeError);
assert.throws(() => new rs.RadixSortGroup({ devices: [0], capacity: 10, topBits: 9 }), /top_bits/);
assert.throws(() => new rs.RadixSortGroup({ devices: [0], capacity: 10, rounds: 17 }), /rounds/);
assert.throws(() => new rs.RadixSortGroup({ devices: [0], capacity: 10, transport: 'tcp' }), TypeError);
assert.throws(() => new rs.RadixSortGroup({ devices: [0], capacity: 2 ** 32 }), /capacity/);
assert.throws(() => rs.addon.groupSort(undefined, [], null, [], null), TypeError);
console.log('node api checks ok');
