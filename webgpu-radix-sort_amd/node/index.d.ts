// Type declarations for the MI355X radix sort's JavaScript API (index.js).  Mirrors the
// reference's exported classes (src/index.ts:1-3) and option shapes.

export declare const GPUBufferUsage: {
  readonly MAP_READ: number; readonly MAP_WRITE: number; readonly COPY_SRC: number;
  readonly COPY_DST: number; readonly INDEX: number; readonly VERTEX: number;
  readonly UNIFORM: number; readonly STORAGE: number; readonly INDIRECT: number;
  readonly QUERY_RESOLVE: number;
};
export declare const GPUMapMode: { readonly READ: number; readonly WRITE: number };

export interface WorkgroupSize { x: number; y: number; }
export interface PlanInfo {
  passes: number; digitBits: number[]; tileKeys: number; gridBlocks: number; workspaceBytes: number;
  /** in-wave stable ranking: lane-ordered LDS atomics, or ballot-match (self-test fallback) */
  rankMode: 'lds_atomic' | 'ballot';
  /** the device's LDS-atomic lane-order self-test: 1 passed, 0 failed, -1 not run */
  laneOrderSelftest: number;
}

export declare class DeviceBuffer {
  readonly device: Device;
  readonly size: number;
  readonly usage: number;
  readonly ptr: bigint | null;
  getMappedRange(offset?: number, size?: number): ArrayBuffer;
  unmap(): void;
  mapAsync(mode: number): Promise<number>;
  destroy(): void;
}

/** rg32uint (key, value) texture: texel (x, y) = record y * width + x, dense in device memory. */
export declare class DeviceTexture extends DeviceBuffer {
  readonly width: number;
  readonly height: number;
  readonly format: 'rg32uint' | 'r32uint';
  readonly bytesPerTexel: number;
}
export interface Extent { width: number; height?: number; }

export declare class QuerySet {
  readonly type: 'timestamp';
  readonly count: number;
  destroy(): void;
}
export interface ComputePassDescriptor {
  timestampWrites?: { querySet: QuerySet; beginningOfPassWriteIndex?: number; endOfPassWriteIndex?: number };
}

export interface ComputePass { end(): void; }
export interface CommandBuffer { readonly commands: ReadonlyArray<() => void>; }
export declare class CommandEncoder {
  beginComputePass(descriptor?: ComputePassDescriptor): ComputePass;
  resolveQuerySet(querySet: QuerySet, firstQuery: number, queryCount: number, destination: DeviceBuffer, destinationOffset?: number): void;
  copyBufferToBuffer(src: DeviceBuffer, srcOffset: number, dst: DeviceBuffer, dstOffset: number, size: number): void;
  copyTextureToBuffer(src: { texture: DeviceTexture }, dst: { buffer: DeviceBuffer; offset?: number; bytesPerRow?: number }, extent: Extent): void;
  finish(): CommandBuffer;
}

export declare class Device {
  constructor(ordinal?: number);
  readonly ordinal: number;
  readonly limits: Readonly<Record<string, number>>;
  readonly queue: {
    submit(commandBuffers: CommandBuffer[]): void;
    writeBuffer(buffer: DeviceBuffer, offset: number, data: ArrayBufferView | ArrayBuffer): void;
    writeTexture(dest: { texture: DeviceTexture }, data: ArrayBufferView | ArrayBuffer, layout: { offset?: number; bytesPerRow?: number }, extent: Extent): void;
    onSubmittedWorkDone(): Promise<void>;
  };
  createBuffer(desc: { size: number; usage?: number; mappedAtCreation?: boolean; label?: string }): DeviceBuffer;
  createQuerySet(desc: { type: 'timestamp'; count: number }): QuerySet;
  createTexture(desc: { size: Extent | [number, number?]; format?: 'rg32uint' | 'r32uint'; usage?: number; label?: string }): DeviceTexture;
  createCommandEncoder(): CommandEncoder;
  synchronize(): void;
  destroy(): void;
}

export declare const gpu: {
  requestAdapter(opts?: { ordinal?: number }): Promise<{ requestDevice(): Promise<Device> } | null>;
};

/** README spelling (README.md:72-88). */
export interface RadixSortKernelOptions {
  device?: Device;
  keys?: DeviceBuffer;
  values?: DeviceBuffer;
  count: number;
  bit_count?: number;
  workgroup_size?: WorkgroupSize;
  check_order?: boolean;
  local_shuffle?: boolean;
  avoid_bank_conflicts?: boolean;
  /** Shipped-source spelling (RadixSortBufferKernel.ts:9-16). */
  data?: { keys: DeviceBuffer; values?: DeviceBuffer };
  bitCount?: number;
  workgroupSize?: WorkgroupSize;
  checkOrder?: boolean;
  localShuffle?: boolean;
  avoidBankConflicts?: boolean;
  /** Digit bits per HBM pass: 0 = auto (8), 2 = the reference's one 4-way split per pass. */
  radixBits?: number;
}

export declare class RadixSortKernel {
  constructor(options: RadixSortKernelOptions);
  readonly buffers: { keys: DeviceBuffer; values?: DeviceBuffer };
  readonly count: number;
  readonly bitCount: number;
  readonly workgroupSize: WorkgroupSize;
  readonly threadsPerWorkgroup: number;
  readonly workgroupCount: number;
  readonly info: PlanInfo;
  /** Records the sort into `pass` (runs at queue.submit) or runs it immediately. */
  dispatch(pass?: ComputePass): void;
  /** Waits for the last sort; throws if a sort failed on the device since the last check. */
  check(): void;
  /** The path the last sort took (waits for it; rs_plan_last_path). */
  lastPath(): "none" | "lsd" | "hybrid" | "hybrid_fallback" | "in_order" | "presorted";
  /** How deep the last hybrid sort split over-full 16-bit buckets: 0, 2 or 3 (rs_plan_last_split). */
  lastSplit(): 0 | 2 | 3;
  destroy(): void;
}
export declare class RadixSortBufferKernel extends RadixSortKernel {}

/** RadixSortTextureKernel.ts:15-35: sorts an rg32uint (key, value) texture in place by key. */
export interface RadixSortTextureKernelOptions {
  device?: Device;
  data?: { texture: DeviceTexture };
  texture?: DeviceTexture;
  count?: number;
  bitCount?: number; bit_count?: number;
  workgroupSize?: WorkgroupSize; workgroup_size?: WorkgroupSize;
  checkOrder?: boolean; check_order?: boolean;
  avoidBankConflicts?: boolean; avoid_bank_conflicts?: boolean;
  radixBits?: number;
}
export declare class RadixSortTextureKernel {
  constructor(options: RadixSortTextureKernelOptions);
  readonly textures: { read: DeviceTexture };
  readonly hasValues: true;
  readonly count: number;
  readonly info: PlanInfo;
  dispatch(pass?: ComputePass): void;
  check(): void;
  lastPath(): "none" | "lsd" | "hybrid" | "hybrid_fallback" | "in_order" | "presorted";
  lastSplit(): 0 | 2 | 3;
  destroy(): void;
}

export declare class PrefixSumKernel {
  constructor(options: { device?: Device; data: DeviceBuffer; count: number; workgroupSize?: WorkgroupSize; avoidBankConflicts?: boolean });
  /** Indirect when dispatchSizeBuffer is given (PrefixSumKernel.ts:147-158). */
  dispatch(pass?: ComputePass, dispatchSizeBuffer?: DeviceBuffer, offset?: number): void;
  getDispatchChain(): number[];
  /** Throws if a scan since the last check failed on the device (timed-out look-back wait). */
  check(): void;
  destroy(): void;
}

/** A device range owned by a RadixSortGroup (one rank's slice of the last sort). */
export declare class GroupBuffer {
  readonly device: Device;
  readonly ptr: bigint;
  readonly size: number;
  readonly host: false;
}

/**
 * Multi-GPU sort from one process (no reference counterpart; SURVEY.md §8(b)/(e)): rank r's
 * slice on devices[r]; after sort() + synchronize(), result(r) is rank r's slice of the global
 * stable sorted order.  C ABI: rs_group_create / rs_group_sort / rs_group_result.
 */
export interface RadixSortGroupOptions {
  devices: Array<Device | number>;
  capacity: number;
  hasValues?: boolean;
  transport?: 'rccl' | 'copy';
  topBits?: number;
  rounds?: number;
}
export declare class RadixSortGroup {
  constructor(options: RadixSortGroupOptions);
  readonly devices: Device[];
  readonly world: number;
  readonly hasValues: boolean;
  sort(slices: Array<{ keys: DeviceBuffer | GroupBuffer; values?: DeviceBuffer | GroupBuffer; count?: number }>): void;
  synchronize(): void;
  /** Timing events on every rank from the next sort on (rs_group_set_profiling). */
  setProfiling(enable: boolean): void;
  /** rank's last sort: ms since its start per step, and its off-rank exchange bytes. */
  times(rank: number): { rounds: number; hist16Ms: number; partitionMs: number; roundDoneMs: number[];
                         regionSortedMs: number[]; doneMs: number; bytesSent: number; bytesRecv: number };
  result(rank: number): { keys: GroupBuffer; values: GroupBuffer | null; count: number };
  results(): Array<{ keys: GroupBuffer; values: GroupBuffer | null; count: number }>;
  destroy(): void;
}
