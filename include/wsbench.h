/* wsbench.h — synthetic workloads and the streaming-copy ceiling for bench.py and
 * the GPU tests (libwsbench.so, benchsupport/).  NOT part of the codec's C ABI
 * (include/wsgpu.h): no reference interface corresponds to these, and the product
 * library libwsgpu.so does not contain them.
 *
 * All pointers are device pointers; work is enqueued on `stream` (a hipStream_t,
 * NULL = the null stream) of HIP device `device` and the calls return without
 * synchronising.  Return 0 on success, else a wsg_api_status code (wsgpu.h). */
#ifndef WSBENCH_H
#define WSBENCH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Fill a device batch of uniform frames: n_frames frames of payload_len bytes,
 * frame k at k*frame_len in wire (frame_len = wsg_encoded_length(payload_len, masked)),
 * opcode/fin/masked as given, payload bytes from splitmix64(seed ^ session) where
 * session = k / frames_per_session; text = 1 generates valid UTF-8 (mixed 1-4 byte
 * code points, ~70% ASCII bytes).  Also fills frame_off and session_first.
 * Byte-identical to the oracle's or_synth_uniform (oracle/ws_oracle.c). */
int wsb_synth_uniform(int device, void* stream, uint64_t seed, uint64_t n_frames, uint32_t payload_len,
                      uint32_t frames_per_session, int opcode, int masked, int text,
                      uint8_t* wire, uint64_t* frame_off, uint32_t* session_first);

/* One frame of a table-driven synthetic batch (wsb_synth_frames): the host
 * plans messages, fragmentation and sessions (benchsupport/synth.py); the device
 * writes headers and payloads.  Message bytes are a pure function of
 * (msg_seed, byte position), so a message cut into fragments at any byte splits
 * its code points across frame boundaries. */
typedef struct wsb_synth_frame {
    uint64_t wire_off;     /* frame start in wire */
    uint64_t msg_seed;     /* message content seed */
    uint32_t payload_len;  /* this fragment's payload length */
    uint32_t msg_pos;      /* offset of this fragment's payload within its message */
    uint32_t msg_len;      /* whole message length */
    uint32_t mask;         /* mask key (little-endian bytes), used when masked */
    int32_t inject_pos;    /* message offset of an injected invalid UTF-8 sequence, -1 = none */
    uint8_t opcode;
    uint8_t flags;         /* bit7 = FIN, bit0 = masked */
    uint8_t text;          /* 1 = valid UTF-8 content (~70% ASCII), 0 = random bytes */
    uint8_t inject_kind;   /* 0: C0 80, 1: ED A0 80, 2: F4 90 80 80, 3: E2 82 'a', 4: FF */
} wsb_synth_frame; /* 40 bytes */

int wsb_synth_frames(int device, void* stream, const wsb_synth_frame* table, uint64_t n_frames, uint8_t* wire);

/* Measured streaming ceiling of this device: best-of-`reps` nontemporal 16-B
 * copy of `bytes` from src to dst, in GB/s of read+write (synchronises). */
int wsb_copy_ceiling(int device, void* stream, const void* src, void* dst, uint64_t bytes, int reps, double* gbs);

#ifdef __cplusplus
}
#endif
#endif /* WSBENCH_H */
