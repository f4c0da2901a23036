'use strict';
// webgpu-radix-sort on MI355X — the reference's JavaScript API over the HIP C ABI.
//
// Exports the reference's classes (src/index.ts:1-3; README.md:61-90):
//   RadixSortKernel / RadixSortBufferKernel  — sort keys (+values) in place, stable, ascending by
//                                              the low bit_count bits
//   PrefixSumKernel                          — in-place exclusive scan
// and a minimal WebGPU-shaped device (gpu.requestAdapter().requestDevice(), createBuffer,
// createCommandEncoder/beginComputePass, queue.submit, mapAsync) so code written for the
// reference runs unchanged: as in WebGPU, dispatch() only RECORDS work into the pass; it runs
// on the device's HIP stream when the command buffer is submitted (AbstractRadixSortKernel.ts:
// 221-247 encode-only; example/tests.ts:78 submit).
//
// All compute is in librsort.so (hand-written gfx950 kernels).  There is no CPU fallback: if
// the addon or the library is missing, require() throws.
//
// Plain ES2019 CommonJS (Node >= 12); types in index.d.ts.

const path = require('path');

const addon = require(path.join(__dirname, 'build', 'rsort_napi.node'));

const GPUBufferUsage = Object.freeze({
  MAP_READ: 0x0001, MAP_WRITE: 0x0002, COPY_SRC: 0x0004, COPY_DST: 0x0008, INDEX: 0x0010,
  VERTEX: 0x0020, UNIFORM: 0x0040, STORAGE: 0x0080, INDIRECT: 0x0100, QUERY_RESOLVE: 0x0200,
});
const GPUMapMode = Object.freeze({ READ: 0x0001, WRITE: 0x0002 });

// ---- device, buffers, command recording -----------------------------------------------------

class DeviceBuffer {
  // A GPUBuffer analogue.  MAP_READ / MAP_WRITE buffers live in host memory (like WebGPU's
  // CPU-visible staging buffers); every other buffer is a HIP device allocation.
  constructor(device, { size, usage = 0, mappedAtCreation = false, label = '' }) {
    if (!(size >= 0)) throw new TypeError('createBuffer: size required');
    this.device = device;
    this.size = size;
    this.usage = usage;
    this.label = label;
    this.host = (usage & (GPUBufferUsage.MAP_READ | GPUBufferUsage.MAP_WRITE)) !== 0;
    this.ptr = this.host ? null : addon.malloc(device.ordinal, Math.max(size, 4));
    this.hostData = this.host ? new ArrayBuffer(size) : null;
    this.mapped = mappedAtCreation ? (this.host ? this.hostData : new ArrayBuffer(size)) : null;
    this.destroyed = false;
  }

  // The whole-buffer range aliases the mapping (writes through it reach the buffer at unmap(),
  // as in WebGPU); a sub-range is returned as a copy.
  getMappedRange(offset = 0, size) {
    if (!this.mapped) throw new Error('buffer is not mapped');
    if (offset === 0 && (size === undefined || size === this.size)) return this.mapped;
    return this.mapped.slice(offset, size === undefined ? undefined : offset + size);
  }

  unmap() {
    if (this.mapped && !this.host) addon.h2d(this.ptr, new Uint8Array(this.mapped), this.device.stream);
    this.mapped = null;
  }

  mapAsync(mode) {
    if (!this.host) return Promise.reject(new Error('mapAsync needs a MAP_READ/MAP_WRITE buffer'));
    try {
      addon.streamSynchronize(this.device.stream);   // results of submitted work are complete
      this.device.checkPlans();                      // and none of them failed on the device
    } catch (e) {
      return Promise.reject(e);
    }
    this.mapped = this.hostData;
    return Promise.resolve(mode);
  }

  destroy() {
    if (!this.destroyed && this.ptr) addon.free(this.ptr);
    this.destroyed = true;
    this.ptr = null;
  }
}

// A GPUTexture analogue for the rg32uint textures of RadixSortTextureKernel: texel (x, y) is the
// 8-byte (key, value) record y * width + x, stored densely row-major in a device allocation
// (RadixSortReorder.ts:42-63 addresses texels exactly this way).
const TEXEL_BYTES = { rg32uint: 8, r32uint: 4 };

class DeviceTexture extends DeviceBuffer {
  constructor(device, { size, format = 'rg32uint', usage = 0, label = '' }) {
    const width = Array.isArray(size) ? size[0] : size.width;
    const height = Array.isArray(size) ? (size[1] || 1) : (size.height || 1);
    const bpt = TEXEL_BYTES[format];
    if (!bpt) throw new TypeError(`createTexture: unsupported format ${format}`);
    super(device, { size: width * height * bpt, usage, label });
    this.width = width;
    this.height = height;
    this.format = format;
    this.bytesPerTexel = bpt;
  }
}

// Timestamp QuerySet (createTimestampQuery, example/tests.ts:247-285): one HIP event per query;
// resolveQuerySet writes nanoseconds relative to the first resolved query, so differences are
// GPU time between the recorded points (timestamps[1] - timestamps[0] in example/index.ts:141).
class QuerySet {
  constructor(device, { type = 'timestamp', count }) {
    if (type !== 'timestamp') throw new TypeError(`createQuerySet: unsupported type ${type}`);
    this.device = device;
    this.type = type;
    this.count = count;
    this.events = Array.from({ length: count }, () => addon.eventCreate());
    this.written = new Array(count).fill(false);
  }
  write(index) {
    addon.eventRecord(this.events[index], this.device.stream);
    this.written[index] = true;
  }
  destroy() {
    for (const e of this.events) if (e) addon.eventDestroy(e);
    this.events = [];
  }
}

class ComputePass {
  constructor(encoder, descriptor) {
    this.encoder = encoder;
    this.timestampWrites = descriptor && descriptor.timestampWrites;
    const tw = this.timestampWrites;
    if (tw && tw.beginningOfPassWriteIndex !== undefined) {
      encoder.commands.push(() => tw.querySet.write(tw.beginningOfPassWriteIndex));
    }
  }
  record(fn) { this.encoder.commands.push(fn); }
  end() {
    const tw = this.timestampWrites;
    if (tw && tw.endOfPassWriteIndex !== undefined) {
      this.encoder.commands.push(() => tw.querySet.write(tw.endOfPassWriteIndex));
    }
  }
}

class CommandEncoder {
  constructor(device) { this.device = device; this.commands = []; }
  beginComputePass(descriptor) { return new ComputePass(this, descriptor); }
  resolveQuerySet(querySet, first, count, dst, dstOffset = 0) {
    const dev = this.device;
    this.commands.push(() => {
      const ts = new BigUint64Array(count);
      const origin = querySet.events[first];
      for (let i = 0; i < count; i += 1) {
        const q = first + i;
        if (!querySet.written[q] || !querySet.written[first]) continue;
        ts[i] = BigInt(Math.round(addon.eventElapsed(origin, querySet.events[q]) * 1e6));
      }
      const bytes = new Uint8Array(ts.buffer);
      if (dst.host) new Uint8Array(dst.hostData, dstOffset, bytes.length).set(bytes);
      else addon.h2d(dst.ptr + BigInt(dstOffset), bytes, dev.stream);
    });
  }
  copyBufferToBuffer(src, srcOffset, dst, dstOffset, size) {
    const dev = this.device;
    this.commands.push(() => {
      if (!src.host && dst.host) {
        addon.streamSynchronize(dev.stream);
        addon.d2h(new Uint8Array(dst.hostData, dstOffset, size), src.ptr + BigInt(srcOffset), dev.stream);
      } else if (src.host && !dst.host) {
        addon.h2d(dst.ptr + BigInt(dstOffset), new Uint8Array(src.hostData, srcOffset, size), dev.stream);
      } else if (!src.host && !dst.host) {
        addon.d2d(dst.ptr + BigInt(dstOffset), src.ptr + BigInt(srcOffset), size, dev.stream);
      } else {
        new Uint8Array(dst.hostData, dstOffset, size).set(new Uint8Array(src.hostData, srcOffset, size));
      }
    });
  }
  // {texture}, {buffer, offset?, bytesPerRow?}, {width, height}: whole rows of a dense texture
  copyTextureToBuffer(src, dst, extent) {
    const tex = src.texture;
    const w = extent.width === undefined ? extent[0] : extent.width;
    const h = (extent.height === undefined ? extent[1] : extent.height) || 1;
    const row = w * tex.bytesPerTexel;
    const pitch = dst.bytesPerRow || row;
    for (let y = 0; y < h; ++y) {
      this.copyBufferToBuffer(tex, y * tex.width * tex.bytesPerTexel, dst.buffer,
        (dst.offset || 0) + y * pitch, row);
    }
  }
  finish() { return { commands: this.commands.slice() }; }
}

class Queue {
  constructor(device) { this.device = device; }
  submit(commandBuffers) {
    for (const cb of commandBuffers) for (const fn of cb.commands) fn();
  }
  // {texture}, data, {offset?, bytesPerRow?}, {width, height}
  writeTexture(dest, data, layout, extent) {
    const tex = dest.texture;
    const bytes = ArrayBuffer.isView(data) ? new Uint8Array(data.buffer, data.byteOffset, data.byteLength)
      : new Uint8Array(data);
    const w = extent.width === undefined ? extent[0] : extent.width;
    const h = (extent.height === undefined ? extent[1] : extent.height) || 1;
    const row = w * tex.bytesPerTexel;
    const pitch = (layout && layout.bytesPerRow) || row;
    const off = (layout && layout.offset) || 0;
    for (let y = 0; y < h; ++y) {
      addon.h2d(tex.ptr + BigInt(y * tex.width * tex.bytesPerTexel),
        bytes.subarray(off + y * pitch, off + y * pitch + row), this.device.stream);
    }
  }
  writeBuffer(buffer, offset, data) {
    const bytes = ArrayBuffer.isView(data) ? new Uint8Array(data.buffer, data.byteOffset, data.byteLength)
      : new Uint8Array(data);
    addon.h2d(buffer.ptr + BigInt(offset), bytes, this.device.stream);
  }
  onSubmittedWorkDone() {
    try {
      addon.streamSynchronize(this.device.stream);
      this.device.checkPlans();
    } catch (e) {
      return Promise.reject(e);
    }
    return Promise.resolve();
  }
}

class Device {
  constructor(ordinal = 0) {
    this.ordinal = ordinal;
    this.stream = null;               // the HIP null stream of this device
    this.queue = new Queue(this);
    // The reference reads these limits (example/tests.ts:10-14, utils.ts:11).
    this.limits = Object.freeze({
      maxComputeWorkgroupsPerDimension: 2147483647,
      maxComputeInvocationsPerWorkgroup: 1024,
      maxComputeWorkgroupSizeX: 1024,
      maxComputeWorkgroupSizeY: 1024,
      maxStorageBufferBindingSize: 2 ** 34,
      maxBufferSize: 2 ** 34,
    });
  }
  // Sort plans created on this device: their device-side failures (rs_plan_check) surface at the
  // synchronising points (mapAsync, onSubmittedWorkDone), as a rejected promise.
  registerPlan(kernel) { (this._plans || (this._plans = new Set())).add(kernel); }
  unregisterPlan(kernel) { if (this._plans) this._plans.delete(kernel); }
  checkPlans() { if (this._plans) for (const k of this._plans) k.check(); }
  createBuffer(desc) { return new DeviceBuffer(this, desc); }
  createTexture(desc) { return new DeviceTexture(this, desc); }
  createQuerySet(desc) { return new QuerySet(this, desc); }
  createCommandEncoder() { return new CommandEncoder(this); }
  synchronize() { addon.streamSynchronize(this.stream); }
  destroy() {}
}

// navigator.gpu-shaped entry point: `await gpu.requestAdapter()` then `requestDevice()`.
const gpu = {
  async requestAdapter(opts = {}) {
    const ordinal = opts.ordinal || 0;
    if (addon.deviceCount() <= ordinal) return null;
    return { async requestDevice() { return new Device(ordinal); } };
  },
};

// ---- kernels ---------------------------------------------------------------------------------

function pick(opts, names, dflt) {
  for (const n of names) if (opts[n] !== undefined && opts[n] !== null) return opts[n];
  return dflt;
}

function bufferPtr(b, name) {
  if (b === undefined || b === null) return null;
  if (typeof b === 'bigint') return b;
  if (b instanceof DeviceBuffer) {
    if (b.host) throw new TypeError(`${name} must be a device (STORAGE) buffer`);
    return b.ptr;
  }
  if (b && typeof b.ptr === 'bigint') return b.ptr;
  throw new TypeError(`${name}: expected a device buffer`);
}

function recordOrRun(pass, fn) {
  if (pass && typeof pass.record === 'function') pass.record(fn);
  else fn();
}

class RadixSortKernel {
  /**
   * Accepts both spellings: README's {device, keys, values, count, check_order, bit_count,
   * workgroup_size, local_shuffle, avoid_bank_conflicts} (README.md:72-88,129,168) and the
   * shipped {device, data: {keys, values}, count, bitCount, workgroupSize, checkOrder,
   * localShuffle, avoidBankConflicts} (RadixSortBufferKernel.ts:9-16, AbstractRadixSortKernel.ts:
   * 14-19, AbstractKernel.ts:3-7).  Defaults: bitCount 32, workgroupSize {x:16,y:16},
   * checkOrder/localShuffle/avoidBankConflicts false (AbstractRadixSortKernel.ts:52-57).
   */
  constructor(options) {
    const opts = options || {};
    const data = opts.data || {};
    this.device = opts.device || null;
    const keys = opts.keys !== undefined ? opts.keys : data.keys;
    const values = opts.values !== undefined ? opts.values : data.values;
    if (keys === undefined || keys === null) throw new TypeError('keys buffer is required');
    this.count = opts.count;
    if (!(this.count >= 0)) throw new TypeError('count is required');
    this.bitCount = pick(opts, ['bit_count', 'bitCount'], 32);
    this.workgroupSize = pick(opts, ['workgroup_size', 'workgroupSize'], { x: 16, y: 16 });
    this.checkOrder = !!pick(opts, ['check_order', 'checkOrder'], false);
    this.localShuffle = !!pick(opts, ['local_shuffle', 'localShuffle'], false);
    this.avoidBankConflicts = !!pick(opts, ['avoid_bank_conflicts', 'avoidBankConflicts'], false);
    this.radixBits = pick(opts, ['radix_bits', 'radixBits'], 0);
    this.buffers = { keys };
    if (values !== undefined && values !== null) this.buffers.values = values;
    this.hasValues = !!this.buffers.values;
    for (const [name, b] of Object.entries(this.buffers)) {
      if (b instanceof DeviceBuffer && b.size < this.count * 4) {
        throw new RangeError(`${name} buffer (${b.size} bytes) smaller than count * 4`);
      }
    }
    this._keys = bufferPtr(keys, 'keys');
    this._values = bufferPtr(this.buffers.values, 'values');
    const flags = (this.hasValues ? addon.FLAG_HAS_VALUES : 0)
      | (this.checkOrder ? addon.FLAG_CHECK_ORDER : 0)
      | (this.localShuffle ? addon.FLAG_LOCAL_SHUFFLE : 0)
      | (this.avoidBankConflicts ? addon.FLAG_AVOID_BANK_CONFLICTS : 0);
    this._plan = addon.planCreate({
      device: this.device ? this.device.ordinal : 0,
      count: this.count,
      bitCount: this.bitCount,
      workgroupX: this.workgroupSize.x,
      workgroupY: this.workgroupSize.y === undefined ? 1 : this.workgroupSize.y,
      flags,
      radixBits: this.radixBits,
    });
    if (this.device && this.device.registerPlan) this.device.registerPlan(this);
  }

  get threadsPerWorkgroup() { return this.workgroupSize.x * (this.workgroupSize.y || 1); }

  /** Wait for the last sort; throws if a sort of this kernel failed on the device since the
   * last check (its output is invalid; rs_plan_check). */
  check() { if (this._plan) addon.planCheck(this._plan); }

  /** The path the last sort took (waits for it): "lsd", "hybrid", "hybrid_fallback", "in_order",
   *  "presorted". */
  lastPath() { return addon.planLastPath(this._plan); }

  /** How deep the last hybrid sort split over-full 16-bit buckets (skewed keys): 0, 2 or 3. */
  lastSplit() { return addon.planLastSplit(this._plan); }

  get workgroupCount() { return Math.ceil(this.count / this.threadsPerWorkgroup); }

  get info() { return addon.planInfo(this._plan); }

  /** Record the sort into `pass` (runs at queue.submit), or run it now when no pass is given. */
  dispatch(pass) {
    const stream = this.device ? this.device.stream : null;
    recordOrRun(pass, () => addon.planSort(this._plan, this._keys, this._values, stream));
  }

  destroy() {
    if (this.device && this.device.unregisterPlan) this.device.unregisterPlan(this);
    if (this._plan) addon.planDestroy(this._plan);
    this._plan = null;
  }
}

class RadixSortBufferKernel extends RadixSortKernel {}

class RadixSortTextureKernel {
  /**
   * {device, data: {texture}, count, bitCount, workgroupSize, checkOrder, avoidBankConflicts}
   * (RadixSortTextureKernel.ts:15-35; README-style snake_case also accepted).  The texture is an
   * rg32uint (key, value) texture from device.createTexture; it is sorted in place by key and
   * always carries values (RadixSortTextureKernel.ts:27-29).
   */
  constructor(options) {
    const opts = options || {};
    const data = opts.data || {};
    this.device = opts.device || null;
    const texture = opts.texture !== undefined ? opts.texture : data.texture;
    if (!(texture instanceof DeviceTexture) && !(texture && typeof texture.ptr === 'bigint')) {
      throw new TypeError('texture is required');
    }
    if (texture.format !== undefined && texture.format !== 'rg32uint') {
      throw new TypeError('texture format must be rg32uint');
    }
    this.count = opts.count !== undefined ? opts.count
      : (texture.width !== undefined ? texture.width * texture.height : undefined);
    if (!(this.count >= 0)) throw new TypeError('count is required');
    if (texture.size !== undefined && texture.size < this.count * 8) {
      throw new RangeError(`texture (${texture.size} bytes) smaller than count * 8`);
    }
    this.bitCount = pick(opts, ['bit_count', 'bitCount'], 32);
    this.workgroupSize = pick(opts, ['workgroup_size', 'workgroupSize'], { x: 16, y: 16 });
    this.checkOrder = !!pick(opts, ['check_order', 'checkOrder'], false);
    this.avoidBankConflicts = !!pick(opts, ['avoid_bank_conflicts', 'avoidBankConflicts'], false);
    this.radixBits = pick(opts, ['radix_bits', 'radixBits'], 0);
    this.textures = { read: texture };
    this._ptr = texture.ptr;
    this._plan = addon.planCreate({
      device: this.device ? this.device.ordinal : 0,
      count: this.count,
      bitCount: this.bitCount,
      workgroupX: this.workgroupSize.x,
      workgroupY: this.workgroupSize.y === undefined ? 1 : this.workgroupSize.y,
      flags: addon.FLAG_INTERLEAVED | (this.checkOrder ? addon.FLAG_CHECK_ORDER : 0)
        | (this.avoidBankConflicts ? addon.FLAG_AVOID_BANK_CONFLICTS : 0),
      radixBits: this.radixBits,
    });
    if (this.device && this.device.registerPlan) this.device.registerPlan(this);
  }

  get hasValues() { return true; }

  check() { if (this._plan) addon.planCheck(this._plan); }

  lastPath() { return addon.planLastPath(this._plan); }

  lastSplit() { return addon.planLastSplit(this._plan); }

  get info() { return addon.planInfo(this._plan); }

  dispatch(pass) {
    const stream = this.device ? this.device.stream : null;
    recordOrRun(pass, () => addon.planSort(this._plan, this._ptr, null, stream));
  }

  destroy() {
    if (this.device && this.device.unregisterPlan) this.device.unregisterPlan(this);
    if (this._plan) addon.planDestroy(this._plan);
    this._plan = null;
  }
}

class PrefixSumKernel {
  /** {device, data, count, workgroupSize, avoidBankConflicts} (PrefixSumKernel.ts:24-43). */
  constructor(options) {
    const opts = options || {};
    this.device = opts.device || null;
    this.data = opts.data;
    this.count = opts.count;
    if (!(this.count >= 0)) throw new TypeError('count is required');
    this.workgroupSize = pick(opts, ['workgroup_size', 'workgroupSize'], { x: 16, y: 16 });
    this.avoidBankConflicts = !!pick(opts, ['avoid_bank_conflicts', 'avoidBankConflicts'], false);
    this._data = bufferPtr(this.data, 'data');
    this._plan = addon.scanPlanCreate(this.device ? this.device.ordinal : 0, this.count,
      this.workgroupSize.x, this.workgroupSize.y === undefined ? 1 : this.workgroupSize.y,
      this.avoidBankConflicts ? addon.FLAG_AVOID_BANK_CONFLICTS : 0);
  }

  /**
   * PrefixSumKernel.ts:147-158.  With dispatchSizeBuffer (a device buffer of u32 (x, y, z)
   * triples, e.g. getDispatchChain() written to it) the dispatch is indirect: the scan runs iff
   * the triple at byte `offset` has no zero entry, decided on the device.
   */
  dispatch(pass, dispatchSizeBuffer, offset = 0) {
    const stream = this.device ? this.device.stream : null;
    if (!dispatchSizeBuffer) {
      recordOrRun(pass, () => addon.scanPlanRun(this._plan, this._data, stream));
      return;
    }
    const buf = bufferPtr(dispatchSizeBuffer, 'dispatchSizeBuffer');
    recordOrRun(pass, () => addon.scanPlanRunIndirect(this._plan, this._data, buf, offset, stream));
  }

  /** PrefixSumKernel.getDispatchChain (PrefixSumKernel.ts:135-137): [x, y, 1] per pipeline. */
  getDispatchChain() { return addon.scanPlanDispatchChain(this._plan); }

  /** Wait for the last dispatch; throws if a scan since the last check failed on the device (a
   * timed-out look-back wait of the single-pass scan: its output is invalid). */
  check() { addon.scanPlanCheck(this._plan); }

  destroy() {
    if (this._plan) addon.scanPlanDestroy(this._plan);
    this._plan = null;
  }
}

// A device range owned by a RadixSortGroup (one rank's slice of the last sort): usable as the
// source of copyBufferToBuffer or as a kernel's keys/values buffer.
class GroupBuffer {
  constructor(device, ptr, size) {
    this.device = device;
    this.ptr = ptr;
    this.size = size;
    this.host = false;
  }
}

class RadixSortGroup {
  /**
   * Multi-GPU sort of an input spread over the GPUs of one node, driven from this one process
   * (the reference has no multi-device path; SURVEY.md §8(b)/(e), BASELINE config 5):
   * {devices: [Device | ordinal, ...], capacity, hasValues = true, transport = 'rccl' | 'copy',
   * topBits = 8, rounds = 4}.  Rank r's slice lives on devices[r].  'rccl' opens one RCCL
   * communicator per device (ncclCommInitAll); 'copy' moves the exchange by peer DMA and also
   * accepts a device listed several times (virtual ranks).
   */
  constructor(options) {
    const opts = options || {};
    const devs = opts.devices;
    if (!Array.isArray(devs) || devs.length === 0) throw new TypeError('devices must be a non-empty array');
    this.devices = devs.map((d) => (d instanceof Device ? d : new Device(d)));
    this.world = this.devices.length;
    this.capacity = opts.capacity;
    if (!(this.capacity >= 0)) throw new TypeError('capacity is required');
    this.hasValues = opts.hasValues === undefined ? true : !!opts.hasValues;
    this._group = addon.groupCreate(this.devices.map((d) => d.ordinal), {
      capacity: this.capacity,
      hasValues: this.hasValues,
      transport: opts.transport || 'rccl',
      topBits: opts.topBits || 0,
      rounds: opts.rounds || 0,
    });
  }

  /**
   * slices: one {keys, values?, count?} per rank (device buffers on devices[r]; count defaults to
   * keys.size / 4).  The inputs are only read.  Runs on each device's stream after the work
   * already submitted there; returns once the exchange sizes are known (the rest is
   * asynchronous: results() after synchronize(), or copies submitted on the devices' queues).
   */
  sort(slices) {
    if (!Array.isArray(slices) || slices.length !== this.world) {
      throw new TypeError(`sort: expected ${this.world} slices`);
    }
    const keys = slices.map((s, r) => bufferPtr(s.keys, `slices[${r}].keys`));
    const values = this.hasValues ? slices.map((s, r) => {
      const v = bufferPtr(s.values, `slices[${r}].values`);
      if (v === null) throw new TypeError(`slices[${r}].values is required (hasValues)`);
      return v;
    }) : null;
    const counts = slices.map((s) => (s.count !== undefined ? s.count : Math.floor(s.keys.size / 4)));
    addon.groupSort(this._group, keys, values, counts, this.devices.map((d) => d.stream));
  }

  /** Wait for the last sort on every device; throws if any of its kernels failed on the device. */
  synchronize() { addon.groupSynchronize(this._group); }

  /** Timing events on every rank from the next sort on (rs_group_set_profiling). */
  setProfiling(enable) { addon.groupSetProfiling(this._group, !!enable); }

  /** Where rank's last sort spent its time (rs_group_times_get; waits for it): ms since the
   * sort's start - hist16Ms, partitionMs, roundDoneMs[], regionSortedMs[], doneMs - and the
   * rank's off-rank exchange bytes (bytesSent, bytesRecv). */
  times(rank) { return addon.groupTimes(this._group, rank); }

  /** Rank r's slice of the global sorted order: {keys, values, count} (group-owned, valid until
   * the next sort or destroy). */
  result(rank) {
    const r = addon.groupResult(this._group, rank);
    const dev = this.devices[rank];
    return {
      keys: new GroupBuffer(dev, r.keys, r.count * 4),
      values: r.values === null ? null : new GroupBuffer(dev, r.values, r.count * 4),
      count: r.count,
    };
  }

  results() { return this.devices.map((_, r) => this.result(r)); }

  destroy() {
    if (this._group) addon.groupDestroy(this._group);
    this._group = null;
  }
}

module.exports = {
  RadixSortGroup,
  GroupBuffer,
  RadixSortKernel,
  RadixSortBufferKernel,
  RadixSortTextureKernel,
  PrefixSumKernel,
  Device,
  DeviceBuffer,
  DeviceTexture,
  QuerySet,
  GPUBufferUsage,
  GPUMapMode,
  gpu,
  addon,
};
