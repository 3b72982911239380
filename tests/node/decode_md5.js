// Decode an Annex-B file through bindings/node/Decoder.js (one NAL per
// decode() call, as Player/mp4.js feeds the wasm decoder) and print one JSON
// line: {"width", "height", "frames": [md5...]}.  A third argument "rgb"
// decodes with {rgb: true} (RGBA pictures).
"use strict";
var fs = require("fs");
var crypto = require("crypto");
var Decoder = require("../../bindings/node/Decoder.js");

var data = new Uint8Array(fs.readFileSync(process.argv[2]));
var starts = [];
for (var i = 0; i + 3 <= data.length; i++) {
  if (data[i] === 0 && data[i + 1] === 0 && data[i + 2] === 1) {
    starts.push(i > 0 && data[i - 1] === 0 ? i - 1 : i);
    i += 2;
  }
}
var out = {width: 0, height: 0, frames: [], infos: 0};
var d = new Decoder({rgb: process.argv[3] === "rgb"});
d.onPictureDecoded = function (buffer, width, height, infos) {
  out.width = width;
  out.height = height;
  if (infos) out.infos += infos.length;
  out.frames.push(crypto.createHash("md5").update(buffer).digest("hex"));
};
for (var k = 0; k < starts.length; k++) {
  var e = k + 1 < starts.length ? starts[k + 1] : data.length;
  d.decode(data.subarray(starts[k], e), {nal: k});
}
d.close();
console.log(JSON.stringify(out));
