// Types of the batch entry (streams-api.mjs) the reference's src/streams-api.ts gains.
export type CompressionFormat = "deflate" | "deflate-raw" | "gzip";
export type DecompressionFormat = CompressionFormat | "deflate64-raw";

export interface BatchOptions {
  /** GPU index (one engine context per device). */
  device?: number;
}
export interface CompressBatchOptions extends BatchOptions {
  /** 1..9, or -1 / undefined for the default (6), as CompressionStream's {level}. Level 0 is not offered by the GPU engine. */
  level?: number;
}
export interface DecompressBatchOptions extends BatchOptions {
  /** Output capacity per stream (bytes), one number for all or one per input. Default max(64 KiB, 16 x input). */
  outCapacity?: number | number[];
}
export type Settled<T> = { status: "fulfilled"; value: T } | { status: "rejected"; reason: Error & { zmsg?: string } };

export function compressBatch(inputs: ArrayBufferView[] | ArrayBuffer[], format?: CompressionFormat,
                              options?: CompressBatchOptions): Promise<Uint8Array[]>;
export function decompressBatch(inputs: ArrayBufferView[] | ArrayBuffer[], format?: DecompressionFormat,
                                options?: DecompressBatchOptions): Promise<Uint8Array[]>;
export function compressBatchSettled(inputs: ArrayBufferView[] | ArrayBuffer[], format?: CompressionFormat,
                                     options?: CompressBatchOptions): Promise<Settled<Uint8Array>[]>;
export function decompressBatchSettled(inputs: ArrayBufferView[] | ArrayBuffer[], format?: DecompressionFormat,
                                       options?: DecompressBatchOptions): Promise<Settled<Uint8Array>[]>;
export function deflateBound(length: number, format?: CompressionFormat): number;
export function engineVersion(): string;
export function selfTest(device?: number): number;
