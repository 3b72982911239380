/* Application-hook probe (tests/test_reference_callers.py): defines the
 * reference's H264SwDecMalloc / H264SwDecFree hooks (inc/H264SwDecApi.h:
 * 160-173) with counters and checks that libh264mi.so allocates and frees its
 * instance through them (reference H264SwDecApi.c:147, :301).  Without a GPU
 * H264SwDecInit fails with MEMFAIL after allocating; with one it succeeds and
 * H264SwDecRelease frees.  Prints "mallocs frees init_ret". */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "H264SwDecApi.h"

static int n_malloc, n_free;

void *H264SwDecMalloc(u32 size) { n_malloc++; return malloc(size); }
void H264SwDecFree(void *ptr) { if (ptr) n_free++; free(ptr); }
void H264SwDecMemcpy(void *dest, void *src, u32 count) { memcpy(dest, src, count); }
void H264SwDecMemset(void *ptr, i32 value, u32 count) { memset(ptr, value, count); }
void H264SwDecTrace(char *s) { (void)s; }

int main(void)
{
    H264SwDecInst inst = NULL;
    H264SwDecRet r = H264SwDecInit(&inst, 0);
    if (r == H264SWDEC_OK) H264SwDecRelease(inst);
    printf("%d %d %d\n", n_malloc, n_free, (int)r);
    return 0;
}
