/* The MB-record format is part of the public C-ABI: include/h264mi_records.h */
#ifndef H264MI_MBREC_INDIRECT_H
#define H264MI_MBREC_INDIRECT_H
#include "../../../include/h264mi_records.h"
#endif
