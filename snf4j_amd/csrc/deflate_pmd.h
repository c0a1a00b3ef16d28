// deflate_pmd.h — PerMessageDeflateEncoder's per-frame decision (PerMessageDeflateEncoder.java
// :55-99 over DeflateEncoder.java:62-104), shared by the device kernels and the CPU harness.
#pragma once
#include <stdint.h>

#include "../../include/wsgpu.h"

#if defined(__HIPCC__)
#define PMD_FN __host__ __device__ inline
#else
#define PMD_FN static inline
#endif

enum { PMD_PASS = 0, PMD_CALL = 1, PMD_EMPTY = 2 };

// One frame: returns PMD_PASS (allowEncoding false: the frame goes on unchanged), PMD_CALL
// (deflate(SYNC_FLUSH) over the payload; the tail 00 00 FF FF is removed from a final
// fragment) or PMD_EMPTY (an empty payload: the deflater is not called and the payload is
// one 00 byte, DeflateEncoder.java:88-93).  *rsv_out: the frame's RSV bits after encoding
// (RSV1 added to TEXT/BINARY, rsvBits :69-79).  *drop: the deflater is discarded after this
// frame (noContext and a final fragment, DeflateEncoder.java:73-76).  Updates compressing
// (:86-98).
PMD_FN int pmd_step(uint8_t* compressing, int opcode, int fin, int rsv, uint32_t len, int no_context,
                    uint8_t* rsv_out, uint8_t* drop) {
    int allow = ((opcode == 1 || opcode == 2) && !(rsv & 4)) || (opcode == 0 && *compressing);
    int kind = PMD_PASS;
    *drop = 0;
    *rsv_out = (uint8_t)rsv;
    if (allow) {
        kind = len ? PMD_CALL : PMD_EMPTY;
        *drop = (uint8_t)(fin && no_context);
        if (opcode == 1 || opcode == 2) *rsv_out = (uint8_t)(rsv | 4);
    }
    if (opcode < 8) {
        if (fin) *compressing = 0;
        else if (!(rsv & 4) && (opcode == 1 || opcode == 2)) *compressing = 1;
    }
    return kind;
}
