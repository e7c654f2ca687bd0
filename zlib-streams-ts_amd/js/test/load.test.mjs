// CPU check: the addon loads, exports its entry points, and without a GPU the
// batch calls fail loudly (no CPU fallback).
import * as api from "../streams-api.mjs";

let ok = 0;
const expect = (c, m) => { if (!c) { console.error("FAIL " + m); process.exit(1); } ok++; };
expect(typeof api.compressBatch === "function", "compressBatch exported");
expect(typeof api.decompressBatch === "function", "decompressBatch exported");
expect(/gfx950/.test(api.engineVersion()), "engine version names gfx950");
expect(api.deflateBound(65536, "deflate-raw") === 65563, "deflateBound raw 64 KiB");
expect(api.deflateBound(262144, "deflate-raw") === 262231, "deflateBound raw 256 KiB");
(async () => {
  let threw = false;
  try { await api.compressBatch([new Uint8Array(10)], "deflate-raw"); } catch (e) { threw = /device|HIP|hip/i.test(String(e.message)); }
  expect(process.env.ZS_EXPECT_GPU ? !threw : threw, "no GPU -> loud failure");
  console.log("ok " + ok);
})().catch((e) => { console.error(e); process.exit(1); });
