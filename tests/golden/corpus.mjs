// Deterministic synthetic corpora (SURVEY.md Appendix B), shared spec with
// tests/corpus.py and zlib-streams-ts_amd/csrc/corpus.cpp.
export function xs(seed) {
  let s = seed >>> 0 || 1;
  return () => { s ^= s << 13; s >>>= 0; s ^= s >>> 17; s ^= s << 5; s >>>= 0; return s; };
}
const VOCAB = ("the of and to in is that for it as was with be by on not he this are or his from at which but have an they you were her she there been one all we their has would when if so no will more can out said up what about its into them than only other new some could time these two may then do first any my now such like our over man me even most made after also did many before must through back years where much your way well down should because each just those people how too little state good very make world still own see men work long get here between both life being under never day same another know while last might us great old year off come since against go came right used take three").split(" ");

export function text(seed, n) {
  const r = xs(seed), out = new Uint8Array(n);
  let o = 0, w = 0;
  while (o < n) {
    const a = r(), idx = Math.min(a % VOCAB.length, (a >>> 12) % VOCAB.length);
    const word = VOCAB[idx];
    for (let i = 0; i < word.length && o < n; i++) out[o++] = word.charCodeAt(i);
    if (o < n) out[o++] = (++w % 13 == 0) ? 10 : 32;
  }
  return out;
}

export function mixed(seed, n) {
  const out = text(seed, n), r = xs((seed ^ 0x85ebca6b) >>> 0);
  for (let k = 0; k + 8192 <= n; k += 8192) for (let j = 0; j < 1024; j++) out[k + 4096 + j] = r() & 0xff;
  return out;
}

export function rand(seed, n) {
  const r = xs(seed), out = new Uint8Array(n);
  for (let i = 0; i < n; i++) out[i] = r() & 0xff;
  return out;
}

// spec: {kind, seed, n, hex}
export function make(spec) {
  switch (spec.kind) {
    case "text": return text(spec.seed >>> 0, spec.n);
    case "mixed": return mixed(spec.seed >>> 0, spec.n);
    case "rand": return rand(spec.seed >>> 0, spec.n);
    case "zeros": return new Uint8Array(spec.n);
    case "ramp": { const o = new Uint8Array(spec.n); for (let j = 0; j < spec.n; j++) o[j] = j % 251; return o; }
    case "hex": return new Uint8Array(Buffer.from(spec.hex, "hex"));
    default: throw new Error("unknown corpus kind " + spec.kind);
  }
}

export const streamSeed = (i) => (0x9e3779b9 ^ i) >>> 0;
