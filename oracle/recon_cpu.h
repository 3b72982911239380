/* ORACLE -- TEST INFRASTRUCTURE ONLY (see recon_cpu.c header). */
#ifndef H264MI_ORACLE_RECON_CPU_H
#define H264MI_ORACLE_RECON_CPU_H

#include <stdint.h>
#include "../broadway_amd/csrc/common/mbrec.h"
#include "../broadway_amd/csrc/host/decoder.h"

#ifdef __cplusplus
extern "C" {
#endif

/* CPU reconstruction backend for the host decoder (tests / CPU baseline) */
H264Backend oracle_backend_create(void);

/* direct access for record-level parity tests */
void    *oracle_ctx_create(int w_mbs, int h_mbs, int nslots);
uint8_t *oracle_ctx_frame(void *ctx, int slot);
int      oracle_recon_picture(void *ctx, const MbRec *rec, const int16_t *coef, int w_mbs, int h_mbs,
                              int cur_slot);
void     oracle_ctx_destroy(void *ctx);

#ifdef __cplusplus
}
#endif

#endif
