// streams-api.mjs -- the batch entry the reference's src/streams-api.ts gains
// (SURVEY.md 8(b)): compressBatch / decompressBatch route whole batches of
// independent streams to the MI355X engine through the N-API addon.
//
// Per stream the result is exactly what piping that buffer alone through
//   new CompressionStream(format, {level})   (src/streams-api.ts -> src/mod/streams.ts:242-251)
//   new DecompressionStream(format)          (src/mod/streams.ts:253-262)
// yields when the whole buffer is written in ONE write() followed by close(),
// including the stream layer's error strings ("init failed: N",
// "process error: N", "finalization error: N", streams.ts:53,117,170).
// The CPU CompressionStream / DecompressionStream classes stay the
// reference's own; this module only adds the batch path.
import { createRequire } from "module";

const require = createRequire(import.meta.url);
const addon = require("./zsnapi.node");

// format -> windowBits exactly as streams.ts:220 (compression) and 233
// (decompression): loose comparisons, and every other value -- unknown strings,
// undefined -- falls through to 15 ("deflate", the zlib wrapper).
const compressWbits = (format) => (format == "gzip" ? 15 + 16 : format == "deflate-raw" ? -15 : 15);
const decompressWbits = (format) =>
  format == "gzip" ? 15 + 16 : format == "deflate-raw" ? -15 : format == "deflate64-raw" ? -16 : 15;
const Z_STREAM_END = 1;
const Z_STREAM_ERROR = -2;
const PHASE_INIT = 1, PHASE_FINISH = 3;

function streamError(status, phase) {
  if (phase === PHASE_INIT) return new Error(`init failed: ${status}`);
  if (phase === PHASE_FINISH) return new Error(`finalization error: ${status}`);
  return new Error(`process error: ${status}`);
}

function checkInputs(inputs) {
  if (!Array.isArray(inputs)) throw new TypeError("inputs must be an array of Uint8Array");
  return inputs.map((x) => {
    if (x instanceof Uint8Array) return x;
    if (ArrayBuffer.isView(x)) return new Uint8Array(x.buffer, x.byteOffset, x.byteLength);
    if (x instanceof ArrayBuffer) return new Uint8Array(x);
    throw new TypeError("inputs must be Uint8Array / ArrayBufferView / ArrayBuffer");
  });
}

// The device set of a batch (SURVEY.md 8(b) "device mask"): options.devices
// (an array of GPU indices: the batch is split into contiguous stream ranges,
// one per GPU, zs_pool) or options.device (one index); default GPU 0.
function devicesOf(options) {
  if (Array.isArray(options.devices)) return options.devices;
  return options.device === undefined ? 0 : options.device;
}

// The addon runs each batch on a worker thread (napi_async_work) and settles a
// Promise: the event loop is not blocked while the GPU works.
async function runCompress(inputs, format, options) {
  options = options || {};
  const wbits = compressWbits(format);
  // streams.ts:221: a level that is not a number means Z_DEFAULT_COMPRESSION (-1 -> 6, deflate.ts:268-270)
  const level = typeof options.level == "number" ? options.level : -1;
  let res;
  try {
    res = await addon.compressBatch(checkInputs(inputs), wbits, level, devicesOf(options));
  } catch (e) {
    // argument validation of deflateInit2_ (deflate.ts:281-294) surfaces as the stream layer's init error
    if (e.code === String(Z_STREAM_ERROR)) throw streamError(Z_STREAM_ERROR, PHASE_INIT);
    throw e;
  }
  return res.outputs.map((out, i) => (res.status[i] === Z_STREAM_END ? out : streamError(res.status[i], PHASE_FINISH)));
}

async function runDecompress(inputs, format, options) {
  options = options || {};
  const wbits = decompressWbits(format);
  const ins = checkInputs(inputs);
  // no outCapacity: unbounded output, as DecompressionStream (streams.ts:46,132-182); a caller cap is a cap
  const res = await addon.decompressBatch(ins, wbits, options.outCapacity, devicesOf(options));
  return res.outputs.map((out, i) => {
    if (res.status[i] === Z_STREAM_END) return out;
    const err = streamError(res.status[i], res.phase[i]);
    err.zmsg = res.message[i];  // the z_stream msg (inflate.ts:397-1031, inffast.ts:108,197,210)
    return err;
  });
}

const settle = (xs) => xs.map((x) => (x instanceof Error ? { status: "rejected", reason: x } : { status: "fulfilled", value: x }));

/** Compress every input as an independent stream; rejects with the first stream's error. */
export async function compressBatch(inputs, format = "deflate", options = {}) {
  const out = await runCompress(inputs, format, options);
  const bad = out.find((x) => x instanceof Error);
  if (bad) throw bad;
  return out;
}

/** Decompress every input as an independent stream; rejects with the first stream's error. */
export async function decompressBatch(inputs, format = "deflate", options = {}) {
  const out = await runDecompress(inputs, format, options);
  const bad = out.find((x) => x instanceof Error);
  if (bad) throw bad;
  return out;
}

/** Per-stream outcomes, Promise.allSettled style. */
export async function compressBatchSettled(inputs, format = "deflate", options = {}) {
  return settle(await runCompress(inputs, format, options));
}

export async function decompressBatchSettled(inputs, format = "deflate", options = {}) {
  return settle(await runDecompress(inputs, format, options));
}

export const deflateBound = (length, format = "deflate") => addon.deflateBound(length, compressWbits(format));

/** Per-stream results with the check value (the reference's strm.adler after the
 * stream: adler32 / crc32 of the uncompressed bytes for "deflate" / "gzip"). */
export async function compressBatchDetailed(inputs, format = "deflate", options = {}) {
  options = options || {};
  const level = typeof options.level == "number" ? options.level : -1;
  return addon.compressBatch(checkInputs(inputs), compressWbits(format), level, devicesOf(options));
}

export async function decompressBatchDetailed(inputs, format = "deflate", options = {}) {
  options = options || {};
  return addon.decompressBatch(checkInputs(inputs), decompressWbits(format), options.outCapacity, devicesOf(options));
}
export const engineVersion = () => addon.version();
export const selfTest = (device = 0) => addon.selfTest(device);
