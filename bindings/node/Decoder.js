// Broadway's Decoder object API (templates/DecoderPost.js:55-301) on the
// MI355X reconstruction path: `require` this module where the emscripten
// Decoder.js was used.
//
//   var Decoder = require('./Decoder.js');
//   var d = new Decoder({});
//   d.onPictureDecoded = function (buffer, width, height, infos) { ... };
//   d.decode(nalU8Array, parInfo);          // synchronous, one NAL per call
//
// buffer: MB-aligned planar I420 (width*height*3/2 bytes, no cropping), or
//         with {rgb: true} RGBA (width*height*4 bytes) converted on the GPU
//         with the per-pixel arithmetic of DecoderPost.js's yuv2rgbcalc.
// infos:  parInfo objects passed since the last picture, stamped with
//         startDecoding / finishDecoding (DecoderPost.js:77-103, :277-281).
// Not supported (outside the reconstruction path): sliceMode.
"use strict";
var path = require("path");
var native = require(process.env.BROADWAY_NATIVE ||
                     path.join(__dirname, "..", "..", "broadway_amd", "lib", "broadway.node"));

function nowValue() {
  var t = process.hrtime();
  return t[0] * 1000 + t[1] / 1e6;
}

function Decoder(parOptions) {
  this.options = parOptions || {};
  if (this.options.sliceMode) {
    throw new Error("sliceMode output is not part of the MI355X path");
  }
  this.infoAr = [];
  this.onPictureDecoded = function (buffer, width, height, infos) {};
  this._h = native.create(0, this.options.rgb ? 1 : 0);
  var self = this;
  this._onPic = function (buffer, width, height) {
    var infos;
    if (self.infoAr.length) {
      infos = self.infoAr;
      infos[0].finishDecoding = nowValue();
    }
    self.infoAr = [];
    self.onPictureDecoded(buffer, width, height, infos);
  };
}

Decoder.prototype.decode = function decode(typedAr, parInfo, copyDoneFun) {
  if (parInfo) {
    this.infoAr.push(parInfo);
    parInfo.startDecoding = nowValue();
  }
  native.decode(this._h, typedAr, this._onPic);
  if (copyDoneFun) copyDoneFun();
};

Decoder.prototype.close = function close() {
  if (this._h) native.release(this._h);
  this._h = null;
};

Decoder.version = native.version();

module.exports = Decoder;
