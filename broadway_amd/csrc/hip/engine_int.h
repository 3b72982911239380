/* engine_int.h -- the engine core's internal interface to the H264Backend
 * adapter (host/hipback.cpp): decoder instances, per-GPU shared engines and
 * the engine / pinned-frame pools.  The adapter is plain host C++ over the
 * HIP runtime API; it touches an engine only through these calls and the
 * public h264mi_engine_* ones (include/h264mi.h).  tests/null_device/
 * implements the same interface (and the HIP calls the adapter makes) on the
 * CPU, so that the adapter's threading runs under TSan / ASan without a GPU.
 * Not part of the C-ABI. */
#ifndef H264MI_ENGINE_INT_H
#define H264MI_ENGINE_INT_H

#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>
#include "../../../include/h264mi.h"

/* one batch of npics host pictures (records + coefficient blocks) onto the
 * engine's stream: staged, uploaded, k_prep + k_wgpp launched; intra_heavy:
 * the launch-shape hint (1 / 0), -1 = derive it from the records */
int engine_decode_host(h264mi_engine *e, int npics, const int *stream, const int *cur_slot,
                       const void *const *recs, const int16_t *const *coefs, const uint32_t *ncoef,
                       int intra_heavy);
/* one host picture whose records and coefficient blocks are in pinned host
 * memory: uploaded straight from them (no staging copy); the caller keeps
 * them unchanged until engine_records_wait returns */
int engine_decode_direct(h264mi_engine *e, int stream, int cur_slot, const void *rec, const int16_t *coef,
                         uint32_t ncoef, int intra_heavy);
/* the last batch's uploads have completed (its host records may change) */
int engine_records_wait(h264mi_engine *e);
/* wait for everything queued on the engine's stream (sleeping when the engine
 * was created under H264MI_BLOCKING_SYNC); no flag accounting */
int engine_wait(h264mi_engine *e);
hipStream_t engine_stream(h264mi_engine *e);
/* a slot's device stride (H264MI_SLOT_BYTES) and its D2H as packed I420 on st */
size_t engine_slot_bytes(const h264mi_engine *e);
int engine_copy_out(h264mi_engine *e, int stream, int slot, uint8_t *dst, hipStream_t st);
/* 1 when H264MI_TEST=1: test hooks are honoured (host/capture.c) */
extern "C" int h264mi_test_hooks(void);
/* device flag words of the batch's pictures (ReconArgs::err), one per picture */
unsigned *engine_err_words(h264mi_engine *e);
/* the engine's shape and whether its waits sleep (H264MI_BLOCKING_SYNC at creation) */
void engine_shape(const h264mi_engine *e, int *w_mbs, int *h_mbs, int *nstreams, int *nslots, int *blocking);
/* an engine without diagnostics state (timing events, profiling buffers) */
int engine_poolable(const h264mi_engine *e);
/* a pooled engine handed to a new decoder instance: settings re-read from the
 * environment, nothing prepped, flags cleared, frames cleared (queued) */
int engine_reuse(h264mi_engine *e);
/* k_conceal's per-MB LDS flags fit this engine's picture size (else the
 * host conceals: h264mi_engine_conceal returns -2) */
int engine_conceal_fits(const h264mi_engine *e);

#endif
