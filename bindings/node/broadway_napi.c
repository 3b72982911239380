/* N-API addon: Broadway's JavaScript Decoder on the MI355X reconstruction
 * path.  A node process `require`s this module in place of the emscripten
 * build (Player/Decoder.js + avc.wasm); bindings/node/Decoder.js wraps it
 * with the DecoderPost.js object API.
 *
 * Native surface (one H264SwDec instance per JS Decoder, unlike the single
 * global instance of the wasm module, Decoder.c:21-25):
 *   create(noOutputReordering, rgb)       -> handle (external); rgb != 0:
 *       pictures arrive as RGBA (width*height*4 bytes), converted on the GPU
 *       (H264SwDecNextPictureRGBA; DecoderPost.js rgb option :82-97)
 *   decode(handle, Uint8Array, onPicture) -> undefined
 *       runs the broadwayDecode loop of Decoder.c:44-162 over the bytes:
 *       HDRS_RDY -> GetInfo; PIC_RDY -> drain NextPicture and call
 *       onPicture(Buffer with a copy of the I420 picture, width, height)
 *       synchronously; after a picture the rest of the
 *       buffer is dropped (Decoder.c:122-134); no end-of-stream flush.
 *   release(handle)
 *   version() -> [major, minor]
 */
#define NAPI_VERSION 4
#include <node_api.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/h264mi.h"

typedef struct {
    H264SwDecInst inst;
    H264SwDecInfo info;
    u32 pic_decode;
    u32 rgb;
    /* rgb mode: the RGBA Buffer the last drain iteration allocated but found
     * no picture for, kept for the next picture instead of thrown away */
    napi_ref spare;
    size_t spare_len;
} JsDec;

#define CHECK(env, call)                                                  \
    do {                                                                  \
        if ((call) != napi_ok) {                                          \
            napi_throw_error((env), NULL, "napi call failed: " #call);    \
            return NULL;                                                  \
        }                                                                 \
    } while (0)

static void finalize_dec(napi_env env, void *data, void *hint)
{
    JsDec *d = (JsDec *)data;
    if (d->spare) napi_delete_reference(env, d->spare);
    if (d->inst) H264SwDecRelease(d->inst);
    free(d);
}

static napi_value js_create(napi_env env, napi_callback_info cbi)
{
    size_t argc = 2;
    napi_value argv[2], out;
    CHECK(env, napi_get_cb_info(env, cbi, &argc, argv, NULL, NULL));
    uint32_t no_reorder = 0, rgb = 0;
    if (argc >= 1) napi_get_value_uint32(env, argv[0], &no_reorder);
    if (argc >= 2) napi_get_value_uint32(env, argv[1], &rgb);
    JsDec *d = (JsDec *)calloc(1, sizeof(JsDec));
    if (!d) { napi_throw_error(env, NULL, "out of memory"); return NULL; }
    if (H264SwDecInit(&d->inst, no_reorder) != H264SWDEC_OK) {
        free(d);
        napi_throw_error(env, NULL, "DECODER INITIALIZATION FAILED");
        return NULL;
    }
    d->pic_decode = 1;
    d->rgb = rgb != 0;
    CHECK(env, napi_create_external(env, d, finalize_dec, NULL, &out));
    return out;
}

static JsDec *get_dec(napi_env env, napi_value v)
{
    void *p = NULL;
    if (napi_get_value_external(env, v, &p) != napi_ok || !p) {
        napi_throw_type_error(env, NULL, "not a decoder handle");
        return NULL;
    }
    return (JsDec *)p;
}

static napi_value js_decode(napi_env env, napi_callback_info cbi)
{
    size_t argc = 3;
    napi_value argv[3], undef;
    CHECK(env, napi_get_cb_info(env, cbi, &argc, argv, NULL, NULL));
    CHECK(env, napi_get_undefined(env, &undef));
    if (argc < 3) { napi_throw_type_error(env, NULL, "decode(handle, bytes, onPicture)"); return NULL; }
    JsDec *d = get_dec(env, argv[0]);
    if (!d || !d->inst) return NULL;
    napi_typedarray_type tt;
    size_t len = 0, off = 0;
    void *data = NULL;
    napi_value ab;
    CHECK(env, napi_get_typedarray_info(env, argv[1], &tt, &len, &data, &ab, &off));
    if (tt != napi_uint8_array) { napi_throw_type_error(env, NULL, "bytes must be a Uint8Array"); return NULL; }
    if (len == 0) return undef;
    /* the decoder modifies its input in place (byte_stream.c:192-232):
     * work on a private copy, as Decoder.js copies into the wasm heap */
    u8 *buf = (u8 *)malloc(len);
    if (!buf) { napi_throw_error(env, NULL, "out of memory"); return NULL; }
    memcpy(buf, data, len);
    H264SwDecInput in;
    H264SwDecOutput out;
    H264SwDecPicture pic;
    memset(&in, 0, sizeof(in));
    in.pStream = buf;
    in.dataLen = (u32)len;
    do {
        in.picId = d->pic_decode;
        H264SwDecRet ret = H264SwDecDecode(d->inst, &in, &out);
        switch ((int)ret) {
        case H264SWDEC_HDRS_RDY_BUFF_NOT_EMPTY:
            if (H264SwDecGetInfo(d->inst, &d->info) != H264SWDEC_OK) { in.dataLen = 0; break; }
            in.dataLen -= (u32)(out.pStrmCurrPos - in.pStream);
            in.pStream = out.pStrmCurrPos;
            break;
        case H264SWDEC_PIC_RDY_BUFF_NOT_EMPTY:
        case H264SWDEC_PIC_RDY:
            in.dataLen = 0;                      /* Decoder.c:130 */
            d->pic_decode++;
            for (;;) {
                const size_t px = (size_t)d->info.picWidth * d->info.picHeight;
                napi_value view, args[3], res;
                if (d->rgb) {
                    /* RGBA straight into a new JS Buffer (DecoderPost.js hands
                     * onPictureDecoded a fresh copy, :89-95) */
                    void *dst = NULL;
                    napi_status st = napi_generic_failure;
                    if (d->spare) {
                        if (d->spare_len == px * 4 && napi_get_reference_value(env, d->spare, &view) == napi_ok && view)
                            st = napi_get_buffer_info(env, view, &dst, NULL);
                        napi_delete_reference(env, d->spare);
                        d->spare = NULL;
                    }
                    if (st != napi_ok && napi_create_buffer(env, px * 4, &dst, &view) != napi_ok) {
                        free(buf);
                        napi_throw_error(env, NULL, "cannot allocate picture buffer");
                        return NULL;
                    }
                    if (H264SwDecNextPictureRGBA(d->inst, &pic, 0, (u8 *)dst) != H264SWDEC_PIC_RDY) {
                        /* no picture: keep the Buffer for the next one */
                        if (napi_create_reference(env, view, 1, &d->spare) == napi_ok) d->spare_len = px * 4;
                        else d->spare = NULL;
                        break;
                    }
                } else {
                    if (H264SwDecNextPicture(d->inst, &pic, 0) != H264SWDEC_PIC_RDY) break;
                    /* the picture is borrowed DPB memory (dpb.c:1443): hand JS a
                     * copy, as SoftAVC.cpp:461-462 does */
                    if (napi_create_buffer_copy(env, px * 3 / 2, pic.pOutputPicture, NULL, &view) != napi_ok) {
                        free(buf);
                        napi_throw_error(env, NULL, "cannot allocate picture buffer");
                        return NULL;
                    }
                }
                args[0] = view;
                napi_create_uint32(env, d->info.picWidth, &args[1]);
                napi_create_uint32(env, d->info.picHeight, &args[2]);
                if (napi_call_function(env, undef, argv[2], 3, args, &res) != napi_ok) {
                    free(buf);
                    return NULL;                 /* JS exception propagates */
                }
            }
            break;
        case H264SWDEC_MEMFAIL:                  /* device allocation failed: no silent fallback */
            free(buf);
            napi_throw_error(env, NULL, "H264SwDecDecode: MEMFAIL (HIP device memory)");
            return NULL;
        default:                                 /* STRM_PROCESSED, errors: buffer consumed */
            in.dataLen = 0;
            break;
        }
    } while (in.dataLen > 0);
    free(buf);
    return undef;
}

static napi_value js_release(napi_env env, napi_callback_info cbi)
{
    size_t argc = 1;
    napi_value argv[1], undef;
    CHECK(env, napi_get_cb_info(env, cbi, &argc, argv, NULL, NULL));
    CHECK(env, napi_get_undefined(env, &undef));
    JsDec *d = argc ? get_dec(env, argv[0]) : NULL;
    if (d && d->inst) {
        H264SwDecRelease(d->inst);
        d->inst = NULL;
    }
    return undef;
}

static napi_value js_version(napi_env env, napi_callback_info cbi)
{
    H264SwDecApiVersion v = H264SwDecGetAPIVersion();
    napi_value arr, a, b;
    CHECK(env, napi_create_array_with_length(env, 2, &arr));
    napi_create_uint32(env, v.major, &a);
    napi_create_uint32(env, v.minor, &b);
    napi_set_element(env, arr, 0, a);
    napi_set_element(env, arr, 1, b);
    return arr;
}

static napi_value init(napi_env env, napi_value exports)
{
    napi_property_descriptor props[] = {
        {"create", NULL, js_create, NULL, NULL, NULL, napi_default, NULL},
        {"decode", NULL, js_decode, NULL, NULL, NULL, napi_default, NULL},
        {"release", NULL, js_release, NULL, NULL, NULL, napi_default, NULL},
        {"version", NULL, js_version, NULL, NULL, NULL, napi_default, NULL},
    };
    napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props);
    return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
