// GPU parity through the JavaScript host path (streams-api.mjs -> zsnapi.node
// -> libzsgpu.so): the reference's golden fixtures (tests/golden/, produced by
// the reference bundle) must come out byte-identical, and failing streams must
// reject with the stream layer's error strings.
import { createHash } from "crypto";
import { readFileSync } from "fs";
import { dirname, join } from "path";
import { fileURLToPath } from "url";
import { MessageChannel } from "worker_threads";

import * as corpus from "../../../tests/golden/corpus.mjs";
import * as api from "../streams-api.mjs";

const here = dirname(fileURLToPath(import.meta.url));
const golden = join(here, "..", "..", "..", "tests", "golden");
const sha = (b) => createHash("sha256").update(b).digest("hex");
let checks = 0;
const expect = (c, m) => { if (!c) throw new Error("FAIL " + m); checks++; };

function deflateCases() {
  const g = JSON.parse(readFileSync(join(golden, "deflate_small.json"), "utf8"));
  const side = JSON.parse(readFileSync(join(golden, "deflate_small_inputs.json"), "utf8"));
  return g.cases.map((c) => ({ c, data: c.spec.kind === "hex_sha" ? new Uint8Array(Buffer.from(side[c.spec.sha256], "hex")) : corpus.make(c.spec) }));
}

function inflateCases() {
  const g = JSON.parse(readFileSync(join(golden, "inflate_small.json"), "utf8"));
  const out = [];
  for (const c of g.cases) {
    if (c.in_hex != null) out.push({ c, data: new Uint8Array(Buffer.from(c.in_hex, "hex")) });
    else if (c.name.startsWith("d64_")) out.push({ c, data: new Uint8Array(readFileSync(join(golden, "d64", c.name.slice(4)))) });
    else if (c.in_len === 0) out.push({ c, data: new Uint8Array(0) });
  }
  return out;
}

async function main() {
  // deflate: every golden case at levels 1..9, batched per (level, format)
  const groups = new Map();
  for (const x of deflateCases()) {
    const k = x.c.level + "/" + x.c.format;
    if (!groups.has(k)) groups.set(k, []);
    groups.get(k).push(x);
  }
  for (const [k, xs] of groups) {
    const [level, format] = k.split("/");
    const outs = await api.compressBatch(xs.map((x) => x.data), format, { level: Number(level) });
    xs.forEach((x, i) => expect(outs[i].length === x.c.out_len && sha(outs[i]) === x.c.out_sha256,
                                `deflate ${k} ${x.c.spec.kind} ${x.c.in_len}`));
  }
  // inflate: KATs, deflate64 fixtures, corrupt streams -> bytes or the reference's error string
  const byFmt = new Map();
  for (const x of inflateCases()) {
    if (!byFmt.has(x.c.format)) byFmt.set(x.c.format, []);
    byFmt.get(x.c.format).push(x);
  }
  for (const [format, xs] of byFmt) {
    const res = await api.decompressBatchSettled(xs.map((x) => x.data), format,
                                                 { outCapacity: xs.map((x) => Math.max(65536, (x.c.out_len || 0) + 4096)) });
    xs.forEach((x, i) => {
      if (x.c.ok) expect(res[i].status === "fulfilled" && sha(res[i].value) === x.c.out_sha256, `inflate ${x.c.name}`);
      else expect(res[i].status === "rejected" && res[i].reason.message === x.c.err, `inflate error ${x.c.name}`);
    });
  }
  // round trip of T-corpus streams in every format
  const inputs = [0, 1, 2, 3].map((i) => corpus.text(corpus.streamSeed(i), 65536));
  for (const format of ["deflate", "deflate-raw", "gzip"]) {
    const back = await api.decompressBatch(await api.compressBatch(inputs, format), format);
    back.forEach((b, i) => expect(Buffer.compare(Buffer.from(b), Buffer.from(inputs[i])) === 0, `round trip ${format} ${i}`));
  }
  // the inputs are copied when the call is made: modifying or transferring (detaching) them before the
  // batch settles changes nothing
  const want = await api.compressBatch(inputs, "deflate-raw");
  const mut = inputs.map((x) => new Uint8Array(x));
  const pm = api.compressBatch(mut, "deflate-raw");
  mut.forEach((x) => x.fill(0x41));
  (await pm).forEach((b, i) => expect(Buffer.compare(Buffer.from(b), Buffer.from(want[i])) === 0, `input modified after the call ${i}`));
  const moved = inputs.map((x) => new Uint8Array(x));
  const pt = api.compressBatch(moved, "deflate-raw");
  const { port1, port2 } = new MessageChannel();
  port1.postMessage(null, moved.map((x) => x.buffer));
  expect(moved[0].length === 0, "transfer detached the input");
  (await pt).forEach((b, i) => expect(Buffer.compare(Buffer.from(b), Buffer.from(want[i])) === 0, `input transferred after the call ${i}`));
  port1.close();
  port2.close();
  // level 0 (deflate_stored) against the reference-made layout goldens
  const l0 = JSON.parse(readFileSync(join(golden, "deflate_level0.json"), "utf8")).cases.filter((c) => c.n <= 300000);
  for (const format of ["deflate", "deflate-raw", "gzip"]) {
    const cs = l0.filter((c) => c.format === format);
    const outs = await api.compressBatch(cs.map((c) => corpus.text(corpus.streamSeed(c.seed_index), c.n)), format, { level: 0 });
    cs.forEach((c, i) => expect(outs[i].length === c.out_len && sha(outs[i]) === c.out_sha256, `level 0 ${format} ${c.n}`));
  }
  // the batch runs on a worker thread: the event loop turns while the GPU works
  let turned = false;
  const big = Array.from({ length: 512 }, (_, i) => corpus.text(corpus.streamSeed(i), 65536));
  const pending = api.compressBatch(big, "deflate-raw", { level: 6 });
  setImmediate(() => { turned = true; });
  await pending;
  expect(turned, "event loop not blocked by a batch");
  // deflateInit2_ validation (deflate.ts:281-294) surfaces as the stream layer's init error
  let msg = "";
  try { await api.compressBatch([inputs[0]], "deflate", { level: 10 }); } catch (e) { msg = e.message; }
  expect(msg === "init failed: -2", "level 10 -> init failed: -2");
  // DecompressionStream has no output cap (streams.ts:46,132-182): default options decode any ratio
  const z64 = new Uint8Array(readFileSync(join(golden, "d64", "zeros_100k.deflate64")));
  const [zout] = await api.decompressBatch([z64], "deflate64-raw");
  expect(zout.length === 100000 && zout.every((b) => b === 0), "zeros_100k.deflate64 with default options");
  const zeros = new Uint8Array(1 << 20);
  for (const format of ["deflate-raw", "deflate", "gzip"]) {
    const [zc] = await api.compressBatch([zeros], format);
    const [zd] = await api.decompressBatch([zc], format);
    expect(zd.length === zeros.length && zd.every((b) => b === 0), `1 MiB of zeros (${zc.length} B) back, ${format}`);
  }
  // an explicit cap is a cap
  const capped = await api.decompressBatchSettled([z64], "deflate64-raw", { outCapacity: 4096 });
  expect(capped[0].status === "rejected", "a caller cap below the output rejects");
  // unknown formats fall through to windowBits 15 and non-number levels to the default (streams.ts:220-221,233)
  const viaBogus = await api.compressBatch(inputs, "bogus");
  const viaDeflate = await api.compressBatch(inputs, "deflate");
  viaBogus.forEach((b, i) => expect(Buffer.compare(Buffer.from(b), Buffer.from(viaDeflate[i])) === 0, `"bogus" == "deflate" ${i}`));
  const backBogus = await api.decompressBatch(viaDeflate, "bogus");
  backBogus.forEach((b, i) => expect(Buffer.compare(Buffer.from(b), Buffer.from(inputs[i])) === 0, `decompress "bogus" ${i}`));
  const viaString = await api.compressBatch(inputs, "deflate-raw", { level: "9" });
  const viaDefault = await api.compressBatch(inputs, "deflate-raw", { level: 6 });
  viaString.forEach((b, i) => expect(Buffer.compare(Buffer.from(b), Buffer.from(viaDefault[i])) === 0, `level "9" -> default ${i}`));
  // the device set: an explicit [0] is the default device's batch
  const viaDevices = await api.compressBatch(inputs, "gzip", { devices: [0] });
  const viaDevice = await api.compressBatch(inputs, "gzip");
  viaDevices.forEach((b, i) => expect(Buffer.compare(Buffer.from(b), Buffer.from(viaDevice[i])) === 0, `devices [0] ${i}`));
  // check values: strm.adler after the stream
  for (const format of ["deflate-raw", "deflate", "gzip"]) {
    const d = await api.compressBatchDetailed(inputs, format);
    const back = await api.decompressBatchDetailed(d.outputs, format);
    d.outputs.forEach((o, i) => {
      const want = format === "deflate-raw" ? 1 : format === "gzip" ? Buffer.from(o).readUInt32LE(o.length - 8)
                                                                     : Buffer.from(o).readUInt32BE(o.length - 4);
      expect(d.check[i] === want, `compress check ${format} ${i}`);
      expect(back.check[i] === (format === "deflate-raw" ? 0 : want), `decompress check ${format} ${i}`);
    });
  }
  expect(api.selfTest() === 0, "LDS lane-order self-test");
  console.log("ok " + checks);
}

main().catch((e) => { console.error(e.message || e); process.exit(1); });
