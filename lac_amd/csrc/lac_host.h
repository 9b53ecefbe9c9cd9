// lac_host.h -- the host side shared by liblac.so's translation units: the context
// (lac_ctx, include/lac.h), live kernel timing (ProfScope, lac_profile_*), error
// reporting, and the few host entry points one family calls in another.
#pragma once
#include <stdarg.h>
#include <stddef.h>
#include <string>
#include <vector>

#include "lac_dev.h"

// ====================================================================== C-ABI
struct lac_ctx {
    int device = 0, prec = 0, pmf_bits = 32;
    int64_t V = 0, B = 0;
    uint64_t cap_bits = 0, cap_words = 0;
    RowStats *stats = nullptr;
    EncState *enc = nullptr;
    DecState *dec = nullptr;
    TailState *tail = nullptr;          // decoder tail in the reference frame (lac_decode_tail_*)
    uint64_t *planeA = nullptr, *planeC = nullptr, *nbits = nullptr;
    uint64_t *own_planeA = nullptr, *own_nbits = nullptr;   // planeA / nbits unless lac_set_output redirects them
    const uint8_t *dbits = nullptr;
    uint64_t dstride = 0;
    const uint64_t *dnbits = nullptr;
    int mode = 0;                       // 0 encode, 1 decode
    int finished = 0;                   // nbits / planeA hold finished streams (a job, lac_encode_finish)
    int open = 0;                       // streams hold coded symbols since the last reset and are not
                                        // finished: their output is split between calls (lac_set_output refuses)
    const uint64_t *fin_planeA = nullptr, *fin_nbits = nullptr;   // where the last finished job was written
    int path = LAC_PATH_AUTO;           // encode kernel path (lac_set_option)
    int64_t fused_min_streams = 2048;   // AUTO: fused kernel from this many streams
    int64_t chunk_steps = 64;           // split path: steps per row-stats launch
    int dpath = LAC_PATH_AUTO;          // decode kernel path
    int64_t wave_decode_min_streams = 2048;   // measured: the stats path wins at 1024 streams
    int fine_decode = 1;                // one-wave decode: per-iteration totals (k_decode_wave_fine)
    int dec_stop = 0;                   // LAC_OPT_DECODE_STOP: stop before the first undetermined symbol
    int64_t block_decode_min_streams = 1536;  // AUTO below wave_decode_min_streams: block path from here
                                              // (measured after the serial-step rework: the stats path wins
                                              // at 4-128 and 288-1024 streams, block at 160-256 -- its
                                              // 16-wave groups fill the chip in one round up to 256
                                              // streams -- and at 1536; profiles/r01/decode_paths_v2/)
    int64_t block_window_lo = 160, block_window_hi = 256;   // AUTO: block path inside this window too --
                                              // one 16-wave group per stream fills the chip in one round
                                              // while streams <= CUs; set from the CU count at open
    int block_waves = 0;                // block path waves per stream (0 = by stream count)
    int mapping = LAC_MAP_CEIL;         // symbol_to_range flavour (lac_set_option)
    int term = LAC_TERM_FLUSH;          // stream termination flavour
    int cus = 256;                      // compute units (persistent grids)
    int q1_shape = 0;                   // logits stats block shape (0 auto; lac_set_option tuning)
    uint64_t *q1chunks = nullptr;       // logits / stats-path decode: [chunk_steps * B][64] chunk totals
    void *dmeta = nullptr;              // stats-path decode: [chunk_steps * B] DecRowMeta
    int64_t *dresume = nullptr;         //                    [B] first step k_decode_lean left
    void *lcdf = nullptr;               // lean decode: [lean_rows][V] per-entry CDF (entry width)
    uint64_t *lchunk = nullptr;         //              [lean_rows][64] chunk exclusive bounds
    void *lmeta = nullptr;              //              [lean_rows] LeanMeta
    int64_t lean_rows = 0;              //              rows the buffers hold
    int lean_esize = 0;                 //              their entry width (4 / 8 bytes)
    int32_t *dprogress = nullptr;       //              [B] decoder progress for the prefetch helpers
    uint64_t *lwin = nullptr;           //              [B][lwin_stride] the bit streams as big-endian words, zero-padded
    int64_t lwin_words = 0;             //              words lwin holds
    float *q1m = nullptr;               //                [chunk_steps * B] row maxima
    uint64_t *pxch = nullptr;           // paired row stats (shape 19): [2 * cus] maximum words
    int64_t xch_abort = -1;             // word of pxch holding the last row-group launch's abort flag
    // live kernel timing (lac_profile_enable): hipEvent pairs around launches
    bool prof = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_used;   // kernel id, (start, stop)
    size_t ev_next = 0;
};

enum { KID_ROW_STATS = 0, KID_ENCODE = 1, KID_FINISH = 2, KID_DECODE = 3, KID_FUSED = 4, KID_DECODE_WAVE = 5,
       KID_Q1_STATS = 6, KID_Q1_DECODE = 7, KID_COUNT = 8 };
// the stats-path decode (k_dec_stats + k_decode_seq) reports under KID_DECODE

static inline hipEvent_t ev_get(lac_ctx *c) {
    if (c->ev_next == c->ev_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        c->ev_pool.push_back(e);
    }
    return c->ev_pool[c->ev_next++];
}

// Brackets one launch with events on its stream when profiling is on.
struct ProfScope {
    lac_ctx *c;
    int kid;
    hipStream_t st;
    hipEvent_t a = nullptr, b = nullptr;
    ProfScope(lac_ctx *c_, int kid_, hipStream_t st_) : c(c_), kid(kid_), st(st_) {
        if (c->prof && kid >= 0) {
            a = ev_get(c);
            b = ev_get(c);
            if (a && b) (void)hipEventRecord(a, st);
        }
    }
    ~ProfScope() {
        if (c->prof && a && b) {
            (void)hipEventRecord(b, st);
            c->ev_used.push_back({kid, {a, b}});
        }
    }
};

// Error reporting (lac_last_error): the message of the last failing call on this thread.
int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) return fail(LAC_E_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

#define CHECK_LAUNCH() HIPCHK(hipGetLastError())

static inline hipStream_t S(void *s) { return reinterpret_cast<hipStream_t>(s); }

// Encode bookkeeping for lac_set_output / lac_pack_bits: a call that coded symbols leaves the
// streams open; a job or finish closes them and records which buffers hold the result.
static inline void enc_mark_open(lac_ctx *c) {
    c->open = 1;
    c->finished = 0;
}
static inline void enc_mark_finished(lac_ctx *c) {
    c->open = 0;
    c->finished = 1;
    c->fin_planeA = c->planeA;
    c->fin_nbits = c->nbits;
}

// encode family (lac_encode.hip), for the logits path's encode (q1_encode)
int enc_reset_launch(lac_ctx *c, hipStream_t st);
int enc_stats_launch(lac_ctx *c, const int32_t *sym, int64_t t0, int64_t n, uint64_t *trace, hipStream_t st);
int enc_finish_launch(lac_ctx *c, int term, hipStream_t st);
// decode family (lac_decode.hip): the per-chunk-of-steps buffers the stats path and the
// logits decode share
int ensure_chunk_buffers(lac_ctx *c);
// logits family (lac_logits.hip): whether a q1 row-stats shape exists (lac_set_option)
bool q1_shape_live(int sh);
