// Golden-vector generator: runs the REFERENCE's own bundle
// (/root/reference/dist/zlib-streams.min.js, imported in place, never copied)
// under Node in the survey container and writes small fixtures into
// tests/golden/.  Only this container runs it; the GPU box reads the fixtures.
//
// The bundle destructures TransformStream from globalThis, which Node 12 lacks,
// so a synchronous TransformStream stand-in is installed first (streams-shim.mjs).
// Each buffer goes through `new CompressionStream(format,{level})` /
// `new DecompressionStream(format)` as ONE write() followed by close() -- the
// parity contract of SURVEY.md F13.
//
// usage: node gen_golden.mjs small            -> deflate_small.json, inflate_small.json
//        node gen_golden.mjs batch SET K P    -> part P of K of a batch set (see BATCH below)
import "./streams-shim.mjs";
import { CompressionStream, DecompressionStream } from "/root/reference/dist/zlib-streams.min.js";
import { make, text, mixed, streamSeed } from "./corpus.mjs";
import crypto from "crypto";
import fs from "fs";
import path from "path";

const HERE = path.dirname(new URL(import.meta.url).pathname);

function drain(s) {
  const parts = s.readable._drain();
  let n = 0;
  for (const p of parts) n += p.length;
  const out = new Uint8Array(n);
  let o = 0;
  for (const p of parts) { out.set(p, o); o += p.length; }
  return out;
}

export function compress(format, level, input) {
  const s = new CompressionStream(format, { level });
  s.writable.write(input);
  s.writable.close();
  return drain(s);
}

export function decompress(format, input) {
  // returns {ok, out, err}; the stream layer throws "process error: N" /
  // "finalization error: N" (streams.ts:117,170)
  const s = new DecompressionStream(format);
  try {
    if (input.length) s.writable.write(input);
    s.writable.close();
    return { ok: true, out: drain(s), err: "" };
  } catch (e) {
    return { ok: false, out: drain(s), err: String(e.message) };
  }
}

const sha = (b) => crypto.createHash("sha256").update(b).digest("hex");
const FORMATS = ["deflate-raw", "deflate", "gzip"];

function smallInputs() {
  const specs = [
    { kind: "hex", hex: "" },
    { kind: "hex", hex: "68656c6c6f" },
    { kind: "hex", hex: "61" },
    { kind: "hex", hex: "6161" },
    { kind: "hex", hex: "616161" },
    { kind: "zeros", n: 258 },
    { kind: "zeros", n: 259 },
    { kind: "zeros", n: 65536 },
    { kind: "zeros", n: 100000 },
    { kind: "ramp", n: 70000 },
    { kind: "rand", seed: 7, n: 1000 },
    { kind: "rand", seed: 8, n: 65536 },
    { kind: "rand", seed: 9, n: 40000 },
    { kind: "text", seed: streamSeed(0), n: 777 },
    { kind: "text", seed: streamSeed(0), n: 65536 },
    { kind: "text", seed: streamSeed(1), n: 32768 },
    { kind: "text", seed: streamSeed(2), n: 32769 },
    { kind: "text", seed: streamSeed(3), n: 65400 },
    { kind: "text", seed: streamSeed(4), n: 70000 },
    { kind: "text", seed: streamSeed(5), n: 131072 },
    { kind: "text", seed: streamSeed(6), n: 200003 },
    { kind: "mixed", seed: streamSeed(0), n: 65536 },
    { kind: "mixed", seed: streamSeed(9), n: 100001 },
    { kind: "mixed", seed: streamSeed(10), n: 262144 },
  ];
  // the slide-schedule corner of SURVEY.md A3: a head candidate at exactly
  // MAX_DIST = 32506 behind position 65274 when the input ends at 65400
  const corner = text(streamSeed(11), 65400);
  corner.set(corner.subarray(32768, 32768 + 20), 65274);
  specs.push({ kind: "hex", hex: Buffer.from(corner).toString("hex"), note: "A3 slide corner n=65400" });
  const corner2 = text(streamSeed(12), 70000);
  corner2.set(corner2.subarray(32768, 32768 + 20), 65274);
  specs.push({ kind: "hex", hex: Buffer.from(corner2).toString("hex"), note: "A3 corner control n=70000" });
  return specs;
}

function genSmall() {
  const cases = [];
  for (const spec of smallInputs()) {
    const input = make(spec);
    const levels = input.length > 100000 ? [1, 4, 6, 9] : [1, 2, 3, 4, 5, 6, 7, 8, 9];
    for (const level of levels) {
      for (const format of FORMATS) {
        if (input.length > 70000 && format != "deflate-raw") continue;
        const out = compress(format, level, input);
        const rec = { spec: spec.kind == "hex" && spec.hex.length > 64 ? { kind: "hex_sha", sha256: sha(input), note: spec.note } : spec,
                      in_len: input.length, in_sha256: sha(input), level, format, out_len: out.length, out_sha256: sha(out) };
        if (out.length <= 512) rec.out_hex = Buffer.from(out).toString("hex");
        cases.push(rec);
      }
    }
  }
  // the two A3 inputs are stored in full (hex) in a side file, they are not regenerable from a spec
  const side = {};
  for (const spec of smallInputs()) if (spec.kind == "hex" && spec.hex.length > 64) side[sha(make(spec))] = spec.hex;
  fs.writeFileSync(path.join(HERE, "deflate_small.json"), JSON.stringify({ generator: "gen_golden.mjs small", reference: "zlib-streams-ts v1.0.13 dist bundle", cases }, null, 0));
  fs.writeFileSync(path.join(HERE, "deflate_small_inputs.json"), JSON.stringify(side));
  console.log("deflate cases", cases.length);
}

function genInflate() {
  const cases = [];
  const add = (name, format, input) => {
    const r = decompress(format, input);
    const rec = { name, format, in_hex: input.length <= 4096 ? Buffer.from(input).toString("hex") : undefined,
                  in_len: input.length, in_sha256: sha(input), ok: r.ok, err: r.err, out_len: r.out.length, out_sha256: sha(r.out) };
    cases.push(rec);
  };
  // reference KATs (test-inflate9-length-code-285.spec.ts:9-15, test-inflate9-stored-block.spec.ts:14,
  // test-streams-empty-input.ts:32-41)
  add("kat_d64_len285", "deflate64-raw", Buffer.from("4b1cfdff07a3e5030000", "hex"));
  add("kat_deflate_len285", "deflate-raw", Buffer.from("4b1c0500", "hex"));
  add("kat_d64_stored_abc", "deflate64-raw", Buffer.from("000300fcff414243", "hex"));
  add("kat_raw_empty_stream", "deflate-raw", Buffer.from("0300", "hex"));
  add("empty_input_raw", "deflate-raw", Buffer.alloc(0));
  add("empty_input_gzip", "gzip", Buffer.alloc(0));
  // deflate64 fixtures (test/data, copied verbatim into tests/golden/d64/)
  for (const f of fs.readdirSync(path.join(HERE, "d64")).sort()) {
    add("d64_" + f, "deflate64-raw", fs.readFileSync(path.join(HERE, "d64", f)));
  }
  // round trips of reference-compressed data through each decoder
  for (const [fmt, dfmt] of [["deflate-raw", "deflate-raw"], ["deflate", "deflate"], ["gzip", "gzip"], ["deflate-raw", "deflate64-raw"]]) {
    for (const spec of [{ kind: "text", seed: streamSeed(20), n: 65536 }, { kind: "mixed", seed: streamSeed(21), n: 65536 },
                        { kind: "rand", seed: 22, n: 5000 }, { kind: "zeros", n: 70000 }]) {
      const c = compress(fmt, 6, make(spec));
      add(`rt_${dfmt}_${spec.kind}`, dfmt, c);
    }
  }
  // corrupted streams: deterministic bit flips / truncations / garbage
  const base = compress("deflate-raw", 6, text(streamSeed(30), 20000));
  const gzb = compress("gzip", 6, text(streamSeed(31), 20000));
  const zlb = compress("deflate", 6, text(streamSeed(32), 20000));
  let rs = 12345;
  const rnd = () => { rs ^= rs << 13; rs >>>= 0; rs ^= rs >>> 17; rs ^= rs << 5; rs >>>= 0; return rs; };
  for (let k = 0; k < 120; k++) {
    const [src, fmt] = k % 3 == 0 ? [base, "deflate-raw"] : k % 3 == 1 ? [gzb, "gzip"] : [zlb, "deflate"];
    const b = Buffer.from(src);
    const mode = k % 4;
    let mut;
    if (mode == 0) { for (let f = 0; f < 1 + (k % 5); f++) { const p = rnd() % Math.min(b.length, 64 + (k * 37) % b.length); b[p] ^= 1 << (rnd() % 8); } mut = b; }
    else if (mode == 1) mut = b.subarray(0, rnd() % b.length);
    else if (mode == 2) { const p = rnd() % b.length; for (let j = 0; j < 16 && p + j < b.length; j++) b[p + j] = rnd() & 0xff; mut = b; }
    else { const p = rnd() % 40; b[p] ^= 0xff; mut = b; }
    add(`corrupt_${k}_${fmt}_m${mode}`, fmt, mut);
  }
  // the inflate_fast window-wrap defect (inffast.ts:139-147): a >32 KiB
  // compressed raw stream whose reference decode differs from its source
  const big = mixed(streamSeed(40), 1 << 18);
  const bigc = compress("deflate-raw", 6, big);
  const r = decompress("deflate-raw", bigc);
  fs.writeFileSync(path.join(HERE, "inffast_wrap_defect.json"), JSON.stringify({
    source: { kind: "mixed", seed: streamSeed(40), n: 1 << 18 }, compressed_len: bigc.length, compressed_sha256: sha(bigc),
    source_sha256: sha(big), ref_ok: r.ok, ref_out_len: r.out.length, ref_out_sha256: sha(r.out), ref_equals_source: sha(r.out) == sha(big) }));
  fs.writeFileSync(path.join(HERE, "inflate_small.json"), JSON.stringify({ generator: "gen_golden.mjs small", cases }, null, 0));
  console.log("inflate cases", cases.length, "defect repro:", sha(r.out) != sha(big));
}

// Batch sets (SURVEY.md §8(d) C2..C5): per-stream (u32 len, 16-byte sha256 prefix) records.
const BATCH = {
  t64_l6_raw: { gen: text, n: 65536, count: 4096, level: 6, format: "deflate-raw" },
  m64_l6_raw: { gen: mixed, n: 65536, count: 4096, level: 6, format: "deflate-raw" },
  t256_l1_raw: { gen: text, n: 262144, count: 4096, level: 1, format: "deflate-raw" },
  t256_l9_raw: { gen: text, n: 262144, count: 4096, level: 9, format: "deflate-raw" },
  t64_l6_gzip: { gen: text, n: 65536, count: 8192, level: 6, format: "gzip" },
  t256_l6_raw: { gen: text, n: 262144, count: 4096, level: 6, format: "deflate-raw" },
  // the same streams decoded back by the reference's DecompressionStream: the
  // stream layer's call boundaries make its window-wrap copy (inffast.ts:133-147)
  // emit bytes that are not the source for some of them
  t256_l6_raw_dec: { gen: text, n: 262144, count: 4096, level: 6, format: "deflate-raw", decode: true },
};

function genBatchPart(setName, K, P) {
  const set = BATCH[setName];
  const lo = Math.floor((set.count * P) / K), hi = Math.floor((set.count * (P + 1)) / K);
  const rec = Buffer.alloc((hi - lo) * 20);
  for (let i = lo; i < hi; i++) {
    let out = compress(set.format, set.level, set.gen(streamSeed(i), set.n));
    if (set.decode) {
      const d = decompress(set.format, out);
      if (!d.ok) throw new Error("reference decode failed: " + d.err);
      out = d.out;
    }
    rec.writeUInt32LE(out.length, (i - lo) * 20);
    crypto.createHash("sha256").update(out).digest().copy(rec, (i - lo) * 20 + 4, 0, 16);
  }
  fs.writeFileSync(`/tmp/golden_${setName}_${P}.bin`, rec);
}

// Level 0 (deflate_stored, deflate.ts:1140-1279, reachable as {level: 0}): the
// stored-block layout depends on the stream layer's 32 KiB input sub-chunks and
// 64 KiB output buffers, so it is recorded per size: output length and hash, and
// the stored blocks' lengths parsed back from the output.
function storedBlocks(format, out) {
  let p = format == "gzip" ? 10 : format == "deflate" ? 2 : 0;
  const blocks = [];
  for (;;) {
    const hdr = out[p], len = out[p + 1] | (out[p + 2] << 8);
    if ((hdr & 6) != 0) throw new Error("not a stored block");
    blocks.push(len);
    p += 5 + len;
    if (hdr & 1) break;
  }
  return { blocks, end: p };
}
function genLevel0() {
  const sizes = [0, 1, 5, 100, 4096, 32767, 32768, 32769, 65530, 65531, 65535, 65536, 65537, 65540, 70000, 98303,
                 98304, 98305, 131071, 131072, 131073, 163840, 196608, 200003, 262144, 300000, 524288, 1048576, 1048581];
  const cases = [];
  for (const n of sizes) {
    const input = text(streamSeed(50), n);
    for (const format of FORMATS) {
      const out = compress(format, 0, input);
      const { blocks, end } = storedBlocks(format, out);
      cases.push({ n, format, seed_index: 50, out_len: out.length, out_sha256: sha(out), blocks, trailer: out.length - end,
                   out_hex: out.length <= 256 ? Buffer.from(out).toString("hex") : undefined });
    }
  }
  fs.writeFileSync(path.join(HERE, "deflate_level0.json"), JSON.stringify({ generator: "gen_golden.mjs level0",
    reference: "zlib-streams-ts v1.0.13 dist bundle", input: "text(streamSeed(50), n)", cases }, null, 0));
  console.log("level0 cases", cases.length);
}

const [mode, a, b, c] = process.argv.slice(2);
if (mode == "small") { genSmall(); genInflate(); }
else if (mode == "level0") genLevel0();
else if (mode == "batch") genBatchPart(a, +b, +c);
else console.log("usage: node gen_golden.mjs small | level0 | batch SET K P");
