// Types of the batch entry (streams-api.mjs) the reference's src/streams-api.ts gains.
// Formats are strings as in streams.ts:220,233: anything other than the names
// below falls through to "deflate" (windowBits 15), exactly as the reference.
export type CompressionFormat = "deflate" | "deflate-raw" | "gzip";
export type DecompressionFormat = CompressionFormat | "deflate64-raw";

export interface BatchOptions {
  /** One GPU index (default 0). */
  device?: number;
  /** GPU indices: the batch is split into contiguous stream ranges, one per GPU (zs_pool). */
  devices?: number[];
}
export interface CompressBatchOptions extends BatchOptions {
  /** 0..9, or -1 / any non-number for the default (6), as CompressionStream's {level} (streams.ts:221). */
  level?: number;
}
export interface DecompressBatchOptions extends BatchOptions {
  /** Output cap per stream (bytes), one number for all or one per input.  Default: none -- the
   * output is unbounded, as DecompressionStream's; a stream over a given cap rejects. */
  outCapacity?: number | number[];
}
export type Settled<T> = { status: "fulfilled"; value: T } | { status: "rejected"; reason: Error & { zmsg?: string } };

export interface CompressDetail {
  status: Int32Array;
  /** strm.adler after each stream: adler32 ("deflate"), crc32 ("gzip") of the input, 1 for "deflate-raw". */
  check: Uint32Array;
  outputs: Uint8Array[];
}
export interface DecompressDetail extends CompressDetail {
  phase: Int32Array;
  message: string[];
  consumed: Int32Array;
}

export function compressBatch(inputs: ArrayBufferView[] | ArrayBuffer[], format?: string,
                              options?: CompressBatchOptions): Promise<Uint8Array[]>;
export function decompressBatch(inputs: ArrayBufferView[] | ArrayBuffer[], format?: string,
                                options?: DecompressBatchOptions): Promise<Uint8Array[]>;
export function compressBatchSettled(inputs: ArrayBufferView[] | ArrayBuffer[], format?: string,
                                     options?: CompressBatchOptions): Promise<Settled<Uint8Array>[]>;
export function decompressBatchSettled(inputs: ArrayBufferView[] | ArrayBuffer[], format?: string,
                                       options?: DecompressBatchOptions): Promise<Settled<Uint8Array>[]>;
export function compressBatchDetailed(inputs: ArrayBufferView[] | ArrayBuffer[], format?: string,
                                      options?: CompressBatchOptions): Promise<CompressDetail>;
export function decompressBatchDetailed(inputs: ArrayBufferView[] | ArrayBuffer[], format?: string,
                                        options?: DecompressBatchOptions): Promise<DecompressDetail>;
export function deflateBound(length: number, format?: string): number;
export function engineVersion(): string;
export function selfTest(device?: number): number;
