// Golden vectors for the `rgb: true` conversion (SURVEY §8f rank 4), made by
// running the REFERENCE's own code under node in the build container: the
// text of DecoderPost.js is read at run time from /root/reference (nothing
// of it is copied into this repository).
//
// 1. yuv2rgbcalc (DecoderPost.js:514-560), the per-pixel conversion, is
//    evaluated for every one of the 2^24 (y, u, v) inputs; the fixture holds
//    the MD5 of that table (uint32 words, index (y << 16) | (u << 8) | v) and
//    a few entries.
// 2. asmFactory's doit (:420-505), driven the way getAsm (:323-356) does, is
//    run on a formula frame and compared with the table: its (y, u, v) result
//    cache is indexed by byte address with 4-byte entries (:431-452), and
//    init's input size `((lumaSize + chromaSize)|0 + chromaSize)|0` (:396)
//    parses as a bitwise OR, which can place the cache over the input's V
//    plane -- so doit's output depends on the cache's history.  The fixture
//    records how many pixels differ; the MI355X path reproduces the table.
//   node tests/golden/make_rgba_golden.js > tests/golden/rgba_golden.json
"use strict";
const fs = require("fs");
const crypto = require("crypto");

const src = fs.readFileSync("/root/reference/templates/DecoderPost.js", "utf8");
function extract(name) {
  const start = src.indexOf("function " + name + "(");
  let depth = 0;
  for (let i = src.indexOf("{", start); i < src.length; i++) {
    if (src[i] === "{") depth++;
    else if (src[i] === "}") { depth--; if (depth === 0) return src.slice(start, i + 1); }
  }
  throw new Error("no " + name);
}
const yuv2rgbcalc = new Function("imul", "min", "max", "return " + extract("yuv2rgbcalc"))(Math.imul, Math.min, Math.max);
const asmFactory = new Function("return " + extract("asmFactory"))();

const table = new Uint32Array(1 << 24);
for (let y = 0; y < 256; y++)
  for (let u = 0; u < 256; u++)
    for (let v = 0; v < 256; v++) table[(y << 16) | (u << 8) | v] = yuv2rgbcalc(y, u, v) >>> 0;
const md5 = (a) => crypto.createHash("md5").update(Buffer.from(a.buffer, a.byteOffset, a.byteLength)).digest("hex");
const samples = {};
for (const [y, u, v] of [[0, 0, 0], [16, 128, 128], [235, 128, 128], [255, 255, 255], [81, 90, 240], [145, 54, 34], [41, 240, 110]])
  samples[`${y},${u},${v}`] = table[(y << 16) | (u << 8) | v].toString(16);

// doit on a 1920x1088 formula frame (same formula as tests/test_rgba.py)
const w = 1920, h = 1088;
const outSize = w * h * 4, inpSize = w * h * 3 / 2, cacheSize = Math.pow(2, 24) * 4;
let heapSize = Math.pow(2, 24);
while (heapSize < outSize + inpSize + cacheSize) heapSize += Math.pow(2, 24);
const heap = new ArrayBuffer(heapSize);
const m = asmFactory(global, {}, heap);
m.init(w, h);
const inp = new Uint8Array(heap, outSize, inpSize);
for (let r = 0; r < h; r++)
  for (let c = 0; c < w; c++) inp[r * w + c] = (r * 29 + c * 3 + ((r * c) >> 3)) & 255;
for (let k = 0; k < w * h / 4; k++) { inp[w * h + k] = (k * 11 + 5) & 255; inp[w * h + w * h / 4 + k] = (k * 7 + (k >> 4)) & 255; }
const frame = Uint8Array.from(inp);           // before doit (the cache may overwrite it)
m.doit();
const out = new Uint32Array(heap, 0, w * h);
let differ = 0;
for (let r = 0; r < h; r++)
  for (let c = 0; c < w; c++) {
    const k = (r >> 1) * (w / 2) + (c >> 1);
    const want = table[(frame[r * w + c] << 16) | (frame[w * h + k] << 8) | frame[w * h + w * h / 4 + k]];
    if (out[r * w + c] !== want) differ++;
  }

process.stdout.write(JSON.stringify({
  source: "templates/DecoderPost.js yuv2rgbcalc + asmFactory, evaluated under node " + process.version,
  table_md5: md5(table), table_samples: samples,
  doit_1920x1088: {pixels: w * h, differ_from_table: differ, out_md5: md5(out)},
}, null, 1) + "\n");
