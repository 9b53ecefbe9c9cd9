/*
 * lac.h -- C-ABI of liblac.so, the MI355X (gfx950) arithmetic coder.
 *
 * Plain pointers and sizes only; HIP streams are passed as `void *`
 * (a hipStream_t, NULL = the default stream).  Device pointers are
 * caller-owned and borrowed for the duration of the call (decode: for the
 * decode session).  One handle <-> one device; a handle is not thread-safe,
 * independent handles are.
 *
 * Each entry point replaces a piece of the reference's predictor->coder call
 * surface (/root/reference):
 *
 *   lac_open / lac_encode_reset   A_to_bin.__init__ state l=0, h=2^prec-1
 *                                 (arith_code.py:157-164); AC(pred, prec) (:144-155)
 *   lac_encode                    A_to_bin.step/run per symbol (:187-192, :207-211):
 *                                 receive_symbol (:169-175) with
 *                                 CDFPredictor.symbol_to_range/fudged_dist
 *                                 (:83-110) + decide_bit/emit_bit (:176-186),
 *                                 for B independent streams, T steps per call
 *   lac_encode_finish             A_to_bin.flush (:193-202) + bits() carry
 *                                 resolution (:227-246) + group_bits (:336-347)
 *   lac_encoded_lengths /         bytes(group_bits(bits(...))) of measure_compress
 *   lac_copy_bits                 (:401-420): L bits, MSB first, zero padded
 *   lac_flush_digits              the raw digits flush() yields (:193-202)
 *   lac_decode_open               A_from_bin.__init__ (:248-256) over a bitstream
 *   lac_decode_step(s)            A_from_bin.step/run (:264-299, :322-326) with
 *                                 CDFPredictor.val_to_symbol (:94-97); n symbols
 *                                 out per stream (the reference stores no n)
 *
 * Status codes: 0 = OK, negative = error; lac_last_error() describes the last
 * failure on the calling thread.  Per-stream coder errors are sticky and are
 * reported by lac_stream_status (the reference raises AssertionError or hangs):
 *   LAC_E_SYMBOL_RANGE  symbol not in [0, V)       arith_code.py:100-101
 *   LAC_E_ZERO_WIDTH    zero-probability symbol on the unfudged path
 *                       (the reference loops forever)
 *   LAC_E_TABLE         all-zero row, or row total >= 2^64
 *   LAC_E_DECODE_RANGE  decoded range misses the value  arith_code.py:277-278
 *   LAC_E_CAPACITY      stream exceeded capacity_bits
 *   LAC_E_PREC          prec outside [2, 61] or 2^(prec-1) < V
 *   LAC_E_FLUSH_ZERO_WIDTH  A_from_bin.flush met a zero-width candidate symbol
 *                       (the reference raises ZeroDivisionError, arith_code.py:307)
 *   LAC_E_FLUSH_LOOP    A_from_bin.flush emits symbols that leave [l, h]
 *                       unchanged (the reference loops forever, :308-313)
 */
#ifndef LAC_H
#define LAC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct lac_ctx lac_ctx;

enum {
    LAC_OK = 0,
    LAC_E_ARG = -1,
    LAC_E_PREC = -2,
    LAC_E_SYMBOL_RANGE = -3,
    LAC_E_ZERO_WIDTH = -4,
    LAC_E_TABLE = -5,
    LAC_E_DECODE_RANGE = -6,
    LAC_E_CAPACITY = -7,
    LAC_E_HIP = -8,
    LAC_E_STATE = -9,
    LAC_E_FLUSH_ZERO_WIDTH = -10,
    LAC_E_FLUSH_LOOP = -11,
    LAC_E_UNDETERMINED = -12      /* not a failure: with LAC_OPT_DECODE_STOP a stream stopped before
                                     the first symbol its bits do not determine, registers and
                                     counters as they were before that symbol (lac_decode_get_state) */
};

enum {                       /* lac_set_option */
    LAC_OPT_ENCODE_PATH = 1,       /* LAC_PATH_*: which encode kernels run */
    LAC_OPT_FUSED_MIN_STREAMS = 2, /* AUTO picks the fused kernel from this many streams (2048) */
    LAC_OPT_MAPPING = 3,           /* LAC_MAP_*: how a symbol's CDF range maps onto [l, h] */
    LAC_OPT_TERMINATION = 4,       /* LAC_TERM_*: how a stream is closed */
    LAC_OPT_DECODE_PATH = 5,       /* LAC_PATH_*: SPLIT = one 4-wave workgroup per stream and step,
                                      FUSED = one wave per stream, all steps of a call in one launch;
                                      STATS, BLOCK = see LAC_PATH_STATS / LAC_PATH_BLOCK;
                                      AUTO = FUSED from 2048 streams, BLOCK at 5/8 CUs .. CUs streams
                                      (160-256 on MI355X) and from 1536, else STATS */
    LAC_OPT_Q1_SHAPE = 6,          /* logits path row-stats shape: 0 = auto (default), 1..4 / 6 = (waves per
                                      row, vectors/thread, rolling prefetch) (1,4,n) (2,8,n) (4,8,n)
                                      (8,8,n) / (8,8,y), 8 = tiles of (8,8,n), 10 = tiles of a
                                      16-wave (16,16,n) block, 14 = tiles of (16,8) with a
                                      tile-walking prefetch, 15 = 16-wave, 8 vectors/thread in
                                      registers + 8 in LDS (rows <= 16384 vectors; 16 table copies
                                      when the row fits a trimmed last slot, <= 16064 vectors),
                                      17 / 18 = the same register + LDS form with 4 rows of
                                      <= 4096 / 2 rows of <= 8192 vectors per 16-wave block,
                                      19 / 20 / 21 = row groups: a row of > 16384 vectors in
                                      2..16 segments, one per row slot of 1 / 2 / 4 rows per
                                      16-wave block (the forms of 15 / 18 / 17; slots are
                                      numbered across the blocks of an XCD, so a segment count
                                      need not divide the blocks); AUTO picks the form that
                                      fills its slots best (f32 V = 128256: 2 slots of 1 row
                                      per block), 22 = one row of <= 20480 vectors per 8-wave
                                      block, whole in registers (+ LDS slots up to 26112),
                                      23 = groups of such blocks (AUTO where the slot form has
                                      several rows per block: bf16 V = 262144, f32 V = 151936);
                                      5, 7, 9, 11, 12, 13 and 16 are retired (AUTO never took
                                      them) and refused with LAC_E_ARG; identical results,
                                      only speed differs */
    LAC_OPT_DECODE_FINE = 7,       /* one-wave decode (FUSED path): 1 = one total per 64 vectors of
                                      the row, so only 1 KB is re-read after the search (default,
                                      rows <= 131072 u32 / 65536 u64 entries); 0 = <= 64 chunk totals */
    LAC_OPT_BLOCK_WAVES = 8,       /* BLOCK decode path: waves per stream (4, 8, 16; 0 = by stream
                                      count, the default) */
    LAC_OPT_DECODE_STOP = 9        /* 1: a decoding stream stops before the first symbol its bits do
                                      not determine (decide_symbol's ls != hs, arith_code.py:268-273)
                                      with LAC_E_UNDETERMINED, registers unchanged, instead of decoding
                                      on over zero padding; decodes then take the STATS path.  0 =
                                      off (default).  For decoders that stop where the reference's
                                      run(bits, stop=0) stops (lac_amd.coder.A_from_bin) */
};
enum {
    LAC_MAP_CEIL = 0,              /* CDFPredictor.symbol_to_range + fudged_dist (arith_code.py:83-110) */
    LAC_MAP_FLOOR = 1              /* Predictor.symbol_to_range (arith_code.py:69-70) and
                                      ACSampler's Region.map (arithmetic_coding.py:160-168) */
};
enum {
    LAC_TERM_FLUSH = 0,            /* A_to_bin.flush (arith_code.py:193-202) */
    LAC_TERM_ACSAMPLER = 1         /* ACSampler.flush_compress: step(1,2,3) + carry flush
                                      (arithmetic_coding.py:50-56) */
};
enum {
    LAC_PATH_AUTO = 0,             /* fused if streams >= fused_min_streams, else split */
    LAC_PATH_SPLIT = 1,            /* row-stats kernel over all (step, stream) rows + coder kernel */
    LAC_PATH_FUSED = 2,            /* one wave per stream: row scan + coder in one kernel */
    LAC_PATH_STATS = 3,            /* decode only: chunk totals of every (step, stream) row in one
                                      full-chip kernel, then a per-stream sequential kernel that
                                      re-reads one chunk per step */
    LAC_PATH_BLOCK = 4             /* decode only: one 4/8/16-wave workgroup per stream, all steps in
                                      one launch; the other waves stream row t+1 while wave 0 decodes
                                      step t (AUTO at 5/8 CUs .. CUs and 1536-2047 streams; rows <= 512 iterations of
                                      64 16-B vectors, 16-B aligned, else STATS) */
};

/* Library identification and the last error message of this thread. */
const char *lac_version(void);
const char *lac_last_error(void);

/* Create a coder for `streams` independent streams over a `vocab`-symbol
 * alphabet at `prec` bits (arith_code.py:157-162), tables of `pmf_bits` = 32
 * (uint32) or 64 (uint64) entries, each stream holding up to
 * `capacity_bits` output bits.  Allocates all device state on `device`. */
int lac_open(int device, int prec, int64_t vocab, int64_t streams, int pmf_bits,
             uint64_t capacity_bits, lac_ctx **out);
int lac_close(lac_ctx *ctx);

/* Tune a context (LAC_OPT_*); results are identical on every path. */
int lac_set_option(lac_ctx *ctx, int option, int64_t value);

/* Reset every stream to l = 0, h = 2^prec - 1 with an empty output. */
int lac_encode_reset(lac_ctx *ctx, void *stream);

/* Encode `steps` symbols per stream.  Row (t, b) of the integer pmf starts at
 * element t*step_stride + b*stream_stride of pmf_dev (a stride of 0 re-uses
 * one row: a static model); sym_dev is int32 [steps][streams].  trace_dev,
 * when not NULL, receives per (t, b) two uint64 {E, k}: the k >= 0 digits the
 * symbol emitted, as the integer E = sum d_i 2^(k-1-i) (first digit 0..3,
 * the rest 0/1).  Asynchronous on `stream`. */
int lac_encode(lac_ctx *ctx, const void *pmf_dev, int64_t step_stride, int64_t stream_stride,
               const int32_t *sym_dev, int64_t steps, uint64_t *trace_dev, void *stream);

/* One whole job in one call: reset every stream, encode `steps` symbols (as
 * lac_encode), flush and pack (as lac_encode_finish).  The batched counterpart
 * of bytes(group_bits(AC(...).to_bin.bits(symbols))) (arith_code.py:207-246,
 * :401-420).  At >= 2048 streams this is a single kernel launch. */
int lac_encode_job(lac_ctx *ctx, const void *pmf_dev, int64_t step_stride, int64_t stream_stride,
                   const int32_t *sym_dev, int64_t steps, uint64_t *trace_dev, void *stream);

/* Keep each stream's registers but drop its completed output words, so the
 * stream continues in at most 64 bits of its capacity.  For callers that read
 * every symbol's digits from trace_dev (A_to_bin.step/run, arith_code.py:
 * 187-211, which yield digits as they go): after a rebase the packed output of
 * lac_encode_finish holds only the tail, while lac_flush_digits stays exact.
 * Asynchronous on `stream`. */
int lac_encode_rebase(lac_ctx *ctx, void *stream);

/* Flush every stream and resolve carries into packed bytes (asynchronous). */
int lac_encode_finish(lac_ctx *ctx, void *stream);

/* Synchronise `stream`; err_host[streams] / err_step_host[streams] (either may
 * be NULL) receive each stream's sticky status and the step it failed at.
 * Returns the first non-zero stream status, or LAC_OK. */
int lac_stream_status(lac_ctx *ctx, int32_t *err_host, int64_t *err_step_host, void *stream);

/* After lac_encode_finish: synchronise and copy the bit length of each stream. */
int lac_encoded_lengths(lac_ctx *ctx, uint64_t *nbits_host, void *stream);

/* Device view of the encoded streams: stream b's bytes start at
 * bits_dev + b*stride_bytes, nbits_dev[b] bits, MSB first, zero padded. */
int lac_encoded_device(lac_ctx *ctx, const uint8_t **bits_dev, uint64_t *stride_bytes,
                       const uint64_t **nbits_dev);

/* Synchronise and copy stream b's packed bytes to dst_host + b*dst_stride. */
int lac_copy_bits(lac_ctx *ctx, uint8_t *dst_host, uint64_t dst_stride, void *stream);

/* Same, device to device (asynchronous on `stream`). */
int lac_copy_bits_dev(lac_ctx *ctx, uint8_t *dst_dev, uint64_t dst_stride, void *stream);

/* Per-stream bit counts (uint64 [streams]) copied device to device (async). */
int lac_copy_nbits_dev(lac_ctx *ctx, uint64_t *dst_dev, void *stream);

/* The encoded streams packed back to back for the wire (after lac_encode_finish): a
 * header of every stream's bit count in `hdr_bytes` = 2 or 4 bytes each (little
 * endian), then stream b's ceil(nbits_b / 8) bytes (measure_compress's
 * bytes(group_bits(bits())), arith_code.py:401-420) for b = 0, 1, ...; *len_dev
 * (device uint64) receives the total length.  dst_dev holds at least
 * streams * (hdr_bytes + 8 * ceil(capacity_bits / 64)) bytes.  Two small launches,
 * asynchronous on `stream`: the multi-GPU gather's payload (lac_amd.dist).
 * LAC_E_ARG for hdr_bytes = 2 when the context's streams can hold 65536 bits or more
 * (8 * 8 * ceil(capacity_bits / 64) >= 65536: the count would not fit); LAC_E_STATE
 * unless the last encode call finished the streams (lac_encode_job,
 * lac_encode_logits_job, lac_encode_finish) and no decode is open. */
int lac_pack_bits(lac_ctx *ctx, uint8_t *dst_dev, int hdr_bytes, uint64_t *len_dev, void *stream);

/* lac_pack_bits appending to a buffer of several jobs (the gatherer's per-batch
 * outbox, lac_amd.dist.BitstreamGatherer): the packed job is written at byte offset
 * *base_dev of dst_dev (0 when base_dev is NULL; device memory, read by the kernel,
 * so jobs chain without a host round trip), *end_dev (device) receives base + the
 * packed length, and *len_out, when not NULL, the packed length -- len_out may be
 * host memory from lac_host_alloc (its device address), which the host reads once
 * the launch has completed, with no copy.  A job that would pass dst_bytes writes
 * nothing: *end_dev = base and *len_out = UINT64_MAX.  Same refusals as
 * lac_pack_bits. */
int lac_pack_bits_at(lac_ctx *ctx, uint8_t *dst_dev, uint64_t dst_bytes, int hdr_bytes, const uint64_t *base_dev,
                     uint64_t *end_dev, uint64_t *len_out, void *stream);

/* The packing kernel of lac_pack_bits_at over `jobs` finished jobs at once, no
 * context: job j's plane A at planeA_dev + j * plane_stride uint64 words (streams
 * slots of cap_words each: a context's plane A after its job, e.g. buffers
 * lac_set_output gave it) and its bit counts at nbits_dev + j * streams.  The jobs are
 * packed back to back from byte *base_dev (0 when NULL) of dst_dev; ends_dev[j]
 * (device) receives the end of job j and lens_out[j] (when not NULL; host memory from
 * lac_host_alloc allowed) its packed length.  One launch on `device`, asynchronous on
 * `stream`; same header rule and fit test as lac_pack_bits_at, per job. */
int lac_pack_jobs(int device, const uint64_t *planeA_dev, uint64_t plane_stride, const uint64_t *nbits_dev,
                  int64_t jobs, int64_t streams, uint64_t cap_words, uint8_t *dst_dev, uint64_t dst_bytes,
                  int hdr_bytes, const uint64_t *base_dev, uint64_t *ends_dev, uint64_t *lens_out, void *stream);

/* Redirect where the context's encodes write their output: plane A (streams *
 * cap_words + 1 uint64, the packed bytes after the job) and the bit counts (streams
 * uint64), caller-owned device buffers that must outlive their use; NULL, NULL
 * restores the context's own.  Every later call that reads or writes the output
 * (encode, finish, lac_copy_bits*, lac_encoded_*, lac_pack_bits*, lac_decode_open
 * with no bits) uses them, so consecutive jobs can leave their output in separate
 * buffers with no copy (lac_amd.dist.BitstreamGatherer packs a batch of them at once,
 * off the encode's stream).
 * Only between jobs: LAC_E_STATE (nothing changed) while a decode is open, or while the
 * streams hold coded symbols that are not finished -- an lac_encode / lac_encode_logits
 * call (or an lac_encode_set_state with symbols) since the last lac_encode_reset, not yet
 * followed by lac_encode_finish: those streams have written part of their planes to the
 * current buffers, and the finish would carry-add over the new ones.  Redirect before a
 * job's first call (lac_encode_job does its own reset) or after it finished.
 * Afterwards the context counts as finished (lac_pack_bits*) exactly when the new
 * buffers are the ones its last finished job was written to (showing that job again);
 * any other buffers need the next finished job first. */
int lac_set_output(lac_ctx *ctx, uint64_t *planeA_dev, uint64_t *nbits_dev);

/* Pinned host memory mapped into the device's address space, coherent (kernels'
 * stores are visible to the host when the launch completes), zero-filled:
 * *host_out is the host address, *dev_out the address kernels use.  For the few
 * words the host reads back per job (lac_pack_bits_at's len_out). */
int lac_host_alloc(uint64_t bytes, void **host_out, void **dev_out);
int lac_host_free(void *host);

/* Synchronise and copy each stream's coder registers l, h (A_to_bin.l/.h,
 * arith_code.py:161-162); either pointer may be NULL. */
int lac_encoder_registers(lac_ctx *ctx, int64_t *l_host, int64_t *h_host, void *stream);

/* The digits flush() emitted per stream (at most 8): digits_host[streams][8],
 * count_host[streams].  Synchronises. */
int lac_flush_digits(lac_ctx *ctx, int8_t *digits_host, int32_t *count_host, void *stream);

/* Encoder checkpoint / resume.  Everything an encoder holds per stream: its registers
 * and counters (A_to_bin's l, h and emitted bits, arith_code.py:157-163, in the O(1)
 * renormalisation's plane form) and the output words written so far.  get copies
 * them to the host; set restores them into a context of the same prec, vocab,
 * streams and capacity, so a job can stop after any lac_encode call and continue
 * later -- in this process or another -- bit for bit.  planes_host, when not NULL, is
 * [2][streams][cap_words] uint64 (plane A, then plane C; cap_words =
 * ceil(capacity_bits / 64)).  set refuses (LAC_E_ARG, nothing copied) register sets no
 * encoder reaches: l outside [0, 2^(prec+1)), h < l, h - l >= 2^prec, L beyond the
 * capacity, nflush outside [-1, 8] (streams with err set are copied as they are), and
 * planes_host == NULL while a stream has bits written (L > 0: its output words would
 * be whatever the context held); get and set refuse a decoding context (LAC_E_STATE;
 * lac_encode_reset first).  A restored context is not finished: lac_pack_bits needs a
 * lac_encode_finish first.
 * Synchronise `stream`. */
typedef struct lac_enc_state {
    int64_t l, h;
    uint64_t L, wa, wc;
    int64_t nsym;
    int32_t err, nflush;
    int64_t err_step;
    int8_t flush[8];
} lac_enc_state;
int lac_encode_get_state(lac_ctx *ctx, lac_enc_state *host_out, uint64_t *planes_host, void *stream);
int lac_encode_set_state(lac_ctx *ctx, const lac_enc_state *host_in, const uint64_t *planes_host, void *stream);

/* Start decoding: stream b reads nbits_dev[b] bits at bits_dev + b*stride_bytes
 * (bits_dev == NULL: this context's own encoded streams).  The buffers are
 * borrowed until the next lac_decode_open / lac_close.  stride_bytes must be a
 * multiple of 8 and every stream's region readable up to it; a stream with
 * nbits_dev[b] > 8 * stride_bytes fails with a sticky LAC_E_ARG (lac_stream_status)
 * and reads nothing. */
int lac_decode_open(lac_ctx *ctx, const uint8_t *bits_dev, uint64_t stride_bytes,
                    const uint64_t *nbits_dev, void *stream);

/* Decode one symbol per stream from row b at pmf_dev + b*stream_stride. */
int lac_decode_step(lac_ctx *ctx, const void *pmf_dev, int64_t stream_stride,
                    int32_t *sym_out_dev, void *stream);

/* Decode `steps` symbols per stream (rows as in lac_encode); sym_out_dev is
 * int32 [steps][streams]. */
int lac_decode_steps(lac_ctx *ctx, const void *pmf_dev, int64_t step_stride, int64_t stream_stride,
                     int64_t steps, int32_t *sym_out_dev, void *stream);

/* ---- logits path --------------------------------
 * Tables are computed in-kernel from raw logits with the integer-exact "q1"
 * quantiser instead of being read from a pmf in HBM: for each row
 *   m = max_i x_i (NaN ignored),  c = RNE_f32(544 - 32 m),
 *   j_i = sat_u32(fmaf(x_i, 32, c)) capped at 544 (NaN, -inf, negatives -> 0),
 *   q_i = max(1, TAB[544 - j_i] >> (24 - k)),  TAB[i] = round(2^24 e^(-i/32))
 * i.e. softmax to 1/32-nat resolution, gaps clamped at 17 nats
 * (include/lac_q1_table.h; DESIGN.md "logits path"), with
 * k = lac_q1_k(prec, vocab) = min(24, prec - 1 - ceil(log2 vocab)) so that
 * T <= 2^(prec-1) and no row is ever fudged.  It replaces the float64 numpy
 * quantiser of llama_compress.py:24-30 (whose output is platform-dependent)
 * with a rule both the GPU and the C oracle reproduce bit for bit; the coder
 * semantics are those of CDFPredictor + A_to_bin / A_from_bin
 * (arith_code.py:76-110, 156-334).  Logit rows: bf16 (uint16 bit patterns) or
 * f32, 16-byte aligned, vocab and strides (in elements) multiples of 8 (bf16)
 * or 4 (f32).  Requires the CEIL mapping and FLUSH termination. */
#define LAC_LOGITS_BF16 1
#define LAC_LOGITS_F32 2

int lac_q1_k(int prec, int64_t vocab);

/* reset + encode `steps` symbols per stream from logits + finish
 * (logits[t*step_stride + b*stream_stride + i], sym_dev[t*streams + b]). */
int lac_encode_logits_job(lac_ctx *ctx, const void *logits_dev, int logit_type, int64_t step_stride,
                          int64_t stream_stride, const int32_t *sym_dev, int64_t steps, uint64_t *trace_dev,
                          void *stream);

/* Incremental form: encode `steps` more symbols per stream from logits,
 * continuing each stream where the last call (lac_encode_reset, lac_encode or
 * lac_encode_logits) left it; close with lac_encode_finish.  Streams may mix
 * pmf and logits steps (each step's table is exact either way). */
int lac_encode_logits(lac_ctx *ctx, const void *logits_dev, int logit_type, int64_t step_stride,
                      int64_t stream_stride, const int32_t *sym_dev, int64_t steps, uint64_t *trace_dev,
                      void *stream);

/* Decode `steps` symbols per stream (after lac_decode_open) with the tables
 * computed from logits; sym_out_dev[t*streams + b] (-1 after an error). */
int lac_decode_logits_steps(lac_ctx *ctx, const void *logits_dev, int logit_type, int64_t step_stride,
                            int64_t stream_stride, int64_t steps, int32_t *sym_out_dev, void *stream);

/* Rows longer than a CU holds (LAC_OPT_Q1_SHAPE 19 / 20 / 21 / 23, AUTO for e.g. f32 V =
 * 128256) are split over 2..16 row slots of workgroups that exchange each row's
 * maximum, which needs every member resident.  When a member is not (another
 * kernel holds CUs) the waiting ones give up after ~0.1 s, raise the launch's
 * abort flag, and a tiled two-pass launch queued behind it recomputes every row:
 * results are identical either way.  Synchronises `stream`; *aborted = 1 if the
 * last such launch of this context took that path. */
int lac_q1_group_aborted(lac_ctx *ctx, int64_t *aborted, void *stream);

/* Materialise the q1 tables: pmf_out_dev[(t*streams + b)*vocab + i] (uint32). */
int lac_quantize_logits(lac_ctx *ctx, const void *logits_dev, int logit_type, int64_t step_stride,
                        int64_t stream_stride, int64_t steps, uint32_t *pmf_out_dev, void *stream);

/* Synchronise; ndet_host[streams] = how many leading decoded symbols the
 * available bits determine, i.e. how many symbols the reference's bit-serial
 * A_from_bin.run(bits, stop=0) emits (arith_code.py:268-299, :322-326). */
int lac_decode_determined(lac_ctx *ctx, int64_t *ndet_host, void *stream);

/* Decoder registers of one stream, A_from_bin's state (arith_code.py:248-256) in
 * the value form: l, h, the prec-bit value window x (bits at or past the stream's
 * nbits read as 0), pos = index of the next bit to read, symbols decoded, the
 * sticky error, and the determined flag / count of lac_decode_determined. */
typedef struct lac_dec_state {
    int64_t l, h, x;
    uint64_t pos;
    int64_t nsym;
    int32_t err, det;
    int64_t err_step, ndet;
} lac_dec_state;

/* Copy every stream's decoder registers to / from the host (synchronise).  With
 * lac_decode_open (which binds a longer bit buffer) and a host-side update of x
 * for the bits that arrived since, this resumes a decoder: the bit-serial
 * A_from_bin.step(bit) of the reference (arith_code.py:291-298) is built on it
 * (lac_amd.coder).  set_state refuses (LAC_E_ARG, nothing copied) register sets
 * no decoder reaches: l outside [0, 2^(prec+1)), h < l, h - l >= 2^prec, pos < prec
 * (streams with err set are copied as they are).  Not thread-safe with launches
 * on the same context. */
int lac_decode_get_state(lac_ctx *ctx, lac_dec_state *host_out, void *stream);
int lac_decode_set_state(lac_ctx *ctx, const lac_dec_state *host_in, void *stream);

/* ---- decoder tail in the reference's register frame (arith_code.py:248-334) ----
 * A_from_bin holds l, h and the received window [lb, hb] (the bits so far read
 * with 0s / 1s past the end).  lac_decode_tail_begin converts every stream's
 * value-form registers (after its determined symbols: lac_decode_determined ==
 * symbols decoded, else the stream gets LAC_E_STATE) into that frame; then each
 * lac_decode_tail_step runs one step per stream:
 *   LAC_TAIL_DECIDE  decide_symbol + emit_symbol + emit_bit (:268-291) on the
 *                    window: emits the symbol both window ends map to, or
 *                    nothing (undetermined).  Where the window leaves [l, h]
 *                    (foreign or corrupt bits) it reproduces the reference:
 *                    LAC_E_SYMBOL_RANGE naming V for tables (AssertionError
 *                    'unknown symbol'), out-of-range symbols for LAC_MAP_FLOOR
 *                    (the uniform Predictor(n) has no range check).
 *   LAC_TAIL_FLUSH   one iteration of A_from_bin.flush (:300-317): while [l, h]
 *                    is not inside [lb, hb], the candidate of largest overlap
 *                    ratio (CPython float ranking, first maximum kept), emitted
 *                    without renormalisation; once inside, the registers reset
 *                    and the stream reports idle.
 * sym_out_dev[b] (int64: uniform symbols can be negative) and code_out_dev[b]:
 * 0 = a symbol, 1 = nothing (undetermined / flushed), < 0 = the stream's sticky
 * error (LAC_E_SYMBOL_RANGE with sym_out = the symbol named, LAC_E_DECODE_RANGE
 * for emit_symbol's AssertionError :277-278, LAC_E_FLUSH_*).  Row b of the
 * stream's current table at pmf_dev + b*stream_stride (LAC_MAP_CEIL; ignored,
 * may be NULL, for LAC_MAP_FLOOR, whose alphabet is the context's vocab).
 * Asynchronous on `stream`. */
#define LAC_TAIL_DECIDE 0
#define LAC_TAIL_FLUSH 1
typedef struct lac_tail_state {
    int64_t l, h, lb, hb;
    int32_t err, done;
    int64_t still, nsym;      /* flush emits with [l, h] unchanged; symbols emitted */
} lac_tail_state;

int lac_decode_tail_begin(lac_ctx *ctx, void *stream);
int lac_decode_tail_step(lac_ctx *ctx, const void *pmf_dev, int64_t stream_stride, int mode,
                         int64_t *sym_out_dev, int32_t *code_out_dev, void *stream);
/* Copy the tail registers to / from the host (synchronise).  set_state refuses
 * (LAC_E_ARG) h < l, hb < lb or values beyond +-2^62; receive_bit (:264-267) is a
 * host-side update of lb, hb between steps. */
int lac_decode_tail_get_state(lac_ctx *ctx, lac_tail_state *host_out, void *stream);
int lac_decode_tail_set_state(lac_ctx *ctx, const lac_tail_state *host_in, void *stream);

/* ---- predictor-mapped coding (host, no device work) ----------------------------
 * A predictor whose symbol_to_range / val_to_symbol are its own code (the
 * reference's toy Predictor subclasses, e.g. ModifiedMarkov arith_code.py:468-522)
 * has no table for the GPU: its caller evaluates the mapping and these functions
 * do the coder's register arithmetic.  Registers stay within +-2^62 (LAC_E_ARG
 * otherwise); prec in [2, 61].
 *   lac_hc_encode_symbol  receive_symbol's narrowing to [l+lo, l+hi-1] plus the
 *                         decide_bit / emit_bit loop (arith_code.py:169-186):
 *                         the digits emitted (<= 64, int8); lo >= hi is
 *                         LAC_E_ZERO_WIDTH (the reference loops forever)
 *   lac_hc_encode_flush   A_to_bin.flush (:193-202): its digits
 *   lac_hc_decode_emit    emit_symbol (:274-283) on regs = {l, h, lb, hb}
 *                         (LAC_E_DECODE_RANGE when the range misses [lb, hb]),
 *                         then, if renormalise, the emit_bit loop (:284-291) */
int lac_hc_encode_symbol(int prec, int64_t *l, int64_t *h, int64_t lo, int64_t hi, int8_t *digits,
                         int32_t *ndigits);
int lac_hc_encode_flush(int prec, int64_t l, int64_t h, int8_t *digits, int32_t *ndigits);
int lac_hc_decode_emit(int prec, int64_t *regs, int64_t lo, int64_t hi, int renormalise);

/* Live kernel timing: with profiling on, every kernel launch is bracketed by
 * hipEvents recorded on its own stream.  lac_profile_read synchronises and
 * returns, per kernel id (0 row_stats, 1 encode, 2 finish, 3 decode_step,
 * 4 encode_fused, 5 decode_wave, 6 q1_stats, 7 q1_decode; 8 slots), the summed device milliseconds and the launch
 * count; reset != 0 clears. */
int lac_profile_enable(lac_ctx *ctx, int on);
int lac_profile_read(lac_ctx *ctx, double *ms_total /*[8]*/, int64_t *launches /*[8]*/, int reset);

#ifdef __cplusplus
}
#endif
#endif /* LAC_H */
