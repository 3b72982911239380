/* Drop-in header name of the Broadway decoder API (reference
 * Decoder/inc/H264SwDecApi.h): callers written against the reference --
 * DecTestBench.c, TestBenchMultipleInstance.c, SoftAVC.cpp, Decoder.c --
 * compile unchanged against this include directory and link against
 * libh264mi.so.  Every declaration lives in h264mi.h. */
#ifndef H264SWDECAPI_H
#define H264SWDECAPI_H
#include "h264mi.h"
#endif
