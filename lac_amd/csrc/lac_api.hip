// lac_api.hip -- liblac.so's context and bookkeeping entry points (include/lac.h):
// open / close, options, per-stream status and output copies, pinned mapped host
// words, live kernel timing, and the host-side register arithmetic for predictors
// with their own mapping (lac_hc.h).  The kernels live in lac_encode.hip,
// lac_decode.hip and lac_logits.hip.
#include "lac_host.h"

static thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

extern "C" {

const char *lac_version(void) { return LAC_VERSION; }
const char *lac_last_error(void) { return g_err.c_str(); }

int lac_open(int device, int prec, int64_t vocab, int64_t streams, int pmf_bits, uint64_t capacity_bits,
             lac_ctx **out) {
    if (!out) return fail(LAC_E_ARG, "out is NULL");
    *out = nullptr;
    if (prec < 2 || prec > 61) return fail(LAC_E_PREC, "prec %d outside [2, 61]", prec);
    if (vocab < 1 || vocab > (int64_t)1 << 31) return fail(LAC_E_ARG, "vocab %lld outside [1, 2^31]", (long long)vocab);
    if (((int64_t)1 << (prec - 1)) < vocab)
        return fail(LAC_E_PREC, "2^(prec-1) = %lld < vocab %lld (the reference coder cannot progress)",
                    (long long)1 << (prec - 1), (long long)vocab);
    if (streams < 1) return fail(LAC_E_ARG, "streams must be >= 1");
    if (pmf_bits != 32 && pmf_bits != 64) return fail(LAC_E_ARG, "pmf_bits must be 32 or 64");
    if (capacity_bits < 64) capacity_bits = 64;
    HIPCHK(hipSetDevice(device));
    lac_ctx *c = new lac_ctx;
    c->device = device;
    if (hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c->cus < 1)
        c->cus = 256;
    c->block_window_hi = c->cus;                      // 256 on MI355X
    c->block_window_lo = (c->cus * 5) / 8;            // 160 on MI355X (measured, profiles/r01/decode_paths_v2/)
    c->prec = prec;
    c->pmf_bits = pmf_bits;
    c->V = vocab;
    c->B = streams;
    c->cap_bits = capacity_bits;
    c->cap_words = (capacity_bits + 63) / 64 + 1;
    hipError_t e = hipSuccess;
    // split path: steps per row-stats launch, enough rows to fill the chip even for 1 stream
    c->chunk_steps = streams >= 512 ? kChunkSteps : ((32768 / streams + 63) / 64) * 64;
    e = e ? e : hipMalloc(&c->stats, sizeof(RowStats) * c->chunk_steps * streams);
    e = e ? e : hipMalloc(&c->enc, sizeof(EncState) * streams);
    e = e ? e : hipMalloc(&c->dec, sizeof(DecState) * streams);
    e = e ? e : hipMalloc(&c->planeA, sizeof(uint64_t) * (c->cap_words * streams + 1));
    e = e ? e : hipMalloc(&c->planeC, sizeof(uint64_t) * (c->cap_words * streams + 1));
    e = e ? e : hipMalloc(&c->nbits, sizeof(uint64_t) * streams);
    e = e ? e : hipMemset(c->nbits, 0, sizeof(uint64_t) * streams);
    c->own_planeA = c->planeA;
    c->own_nbits = c->nbits;
    if (e != hipSuccess) {
        lac_close(c);
        return fail(LAC_E_HIP, "device allocation: %s", hipGetErrorString(e));
    }
    int rc = lac_encode_reset(c, nullptr);
    if (rc) { lac_close(c); return rc; }
    if ((e = hipDeviceSynchronize()) != hipSuccess) {
        lac_close(c);
        return fail(LAC_E_HIP, "hipDeviceSynchronize: %s", hipGetErrorString(e));
    }
    *out = c;
    return LAC_OK;
}

int lac_close(lac_ctx *c) {
    if (!c) return LAC_OK;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    (void)hipFree(c->stats);
    (void)hipFree(c->enc);
    (void)hipFree(c->dec);
    (void)hipFree(c->tail);
    (void)hipFree(c->own_planeA ? c->own_planeA : c->planeA);
    (void)hipFree(c->planeC);
    (void)hipFree(c->own_nbits ? c->own_nbits : c->nbits);
    (void)hipFree(c->q1chunks);
    (void)hipFree(c->dmeta);
    (void)hipFree(c->dresume);
    (void)hipFree(c->lcdf);
    (void)hipFree(c->lchunk);
    (void)hipFree(c->lmeta);
    (void)hipFree(c->dprogress);
    (void)hipFree(c->lwin);
    (void)hipFree(c->q1m);
    (void)hipFree(c->pxch);
    for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
    delete c;
    return LAC_OK;
}

int lac_set_option(lac_ctx *c, int option, int64_t value) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    switch (option) {
    case LAC_OPT_ENCODE_PATH:
        if (value < LAC_PATH_AUTO || value > LAC_PATH_FUSED) return fail(LAC_E_ARG, "bad encode path %lld", (long long)value);
        c->path = (int)value;
        return LAC_OK;
    case LAC_OPT_FUSED_MIN_STREAMS:
        if (value < 1) return fail(LAC_E_ARG, "fused_min_streams must be >= 1");
        c->fused_min_streams = value;
        return LAC_OK;
    case LAC_OPT_DECODE_PATH:
        if (value < LAC_PATH_AUTO || value > LAC_PATH_BLOCK) return fail(LAC_E_ARG, "bad decode path");
        c->dpath = (int)value;
        return LAC_OK;
    case LAC_OPT_BLOCK_WAVES:
        if (value != 0 && value != 4 && value != 8 && value != 16) return fail(LAC_E_ARG, "block waves: 0, 4, 8 or 16");
        c->block_waves = (int)value;
        return LAC_OK;
    case LAC_OPT_DECODE_STOP:
        if (value != 0 && value != 1) return fail(LAC_E_ARG, "decode_stop must be 0 or 1");
        c->dec_stop = (int)value;
        return LAC_OK;
    case LAC_OPT_DECODE_FINE:
        if (value != 0 && value != 1) return fail(LAC_E_ARG, "decode_fine must be 0 or 1");
        c->fine_decode = (int)value;
        return LAC_OK;
    case LAC_OPT_Q1_SHAPE:
        if (!q1_shape_live((int)value) || value != (int)value) return fail(LAC_E_ARG, "bad or retired q1 shape");
        c->q1_shape = (int)value;
        return LAC_OK;
    case LAC_OPT_MAPPING:
        if (value != LAC_MAP_CEIL && value != LAC_MAP_FLOOR) return fail(LAC_E_ARG, "bad mapping");
        c->mapping = (int)value;
        return LAC_OK;
    case LAC_OPT_TERMINATION:
        if (value != LAC_TERM_FLUSH && value != LAC_TERM_ACSAMPLER) return fail(LAC_E_ARG, "bad termination");
        c->term = (int)value;
        return LAC_OK;
    default:
        return fail(LAC_E_ARG, "unknown option %d", option);
    }
}

int lac_stream_status(lac_ctx *c, int32_t *err_host, int64_t *err_step_host, void *stream) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(S(stream)));
    int first = LAC_OK;
    if (c->mode == 0) {
        std::vector<EncState> v(c->B);
        HIPCHK(hipMemcpy(v.data(), c->enc, sizeof(EncState) * c->B, hipMemcpyDeviceToHost));
        for (int64_t b = 0; b < c->B; b++) {
            if (err_host) err_host[b] = v[b].err;
            if (err_step_host) err_step_host[b] = v[b].err ? v[b].err_step : -1;
            if (!first && v[b].err) first = v[b].err;
        }
    } else {
        std::vector<DecState> v(c->B);
        HIPCHK(hipMemcpy(v.data(), c->dec, sizeof(DecState) * c->B, hipMemcpyDeviceToHost));
        for (int64_t b = 0; b < c->B; b++) {
            if (err_host) err_host[b] = v[b].err;
            if (err_step_host) err_step_host[b] = v[b].err ? v[b].err_step : -1;
            if (!first && v[b].err) first = v[b].err;
        }
    }
    if (first) fail(first, "a stream reported status %d", first);
    return first;
}

int lac_encoded_lengths(lac_ctx *c, uint64_t *nbits_host, void *stream) {
    if (!c || !nbits_host) return fail(LAC_E_ARG, "NULL argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(S(stream)));
    HIPCHK(hipMemcpy(nbits_host, c->nbits, sizeof(uint64_t) * c->B, hipMemcpyDeviceToHost));
    return LAC_OK;
}

int lac_encoded_device(lac_ctx *c, const uint8_t **bits_dev, uint64_t *stride_bytes, const uint64_t **nbits_dev) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    if (bits_dev) *bits_dev = reinterpret_cast<const uint8_t *>(c->planeA);
    if (stride_bytes) *stride_bytes = c->cap_words * 8;
    if (nbits_dev) *nbits_dev = c->nbits;
    return LAC_OK;
}

int lac_copy_bits(lac_ctx *c, uint8_t *dst, uint64_t dst_stride, void *stream) {
    if (!c || !dst || dst_stride == 0) return fail(LAC_E_ARG, "bad argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(S(stream)));
    const uint64_t src_stride = c->cap_words * 8;
    const uint64_t width = dst_stride < src_stride ? dst_stride : src_stride;
    HIPCHK(hipMemcpy2D(dst, dst_stride, c->planeA, src_stride, width, (size_t)c->B, hipMemcpyDeviceToHost));
    return LAC_OK;
}

int lac_copy_bits_dev(lac_ctx *c, uint8_t *dst, uint64_t dst_stride, void *stream) {
    if (!c || !dst || dst_stride == 0) return fail(LAC_E_ARG, "bad argument");
    HIPCHK(hipSetDevice(c->device));
    const uint64_t src_stride = c->cap_words * 8;
    const uint64_t width = dst_stride < src_stride ? dst_stride : src_stride;
    HIPCHK(hipMemcpy2DAsync(dst, dst_stride, c->planeA, src_stride, width, (size_t)c->B, hipMemcpyDeviceToDevice,
                            S(stream)));
    return LAC_OK;
}

int lac_host_alloc(uint64_t bytes, void **host_out, void **dev_out) {
    if (!host_out || !dev_out || bytes == 0) return fail(LAC_E_ARG, "bad argument");
    void *h = nullptr;
    HIPCHK(hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent));
    void *d = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&d, h, 0);
    if (e != hipSuccess) {
        (void)hipHostFree(h);
        return fail(LAC_E_HIP, "hipHostGetDevicePointer: %s", hipGetErrorString(e));
    }
    memset(h, 0, bytes);
    *host_out = h;
    *dev_out = d;
    return LAC_OK;
}

int lac_host_free(void *host) {
    if (host) HIPCHK(hipHostFree(host));
    return LAC_OK;
}

int lac_copy_nbits_dev(lac_ctx *c, uint64_t *dst, void *stream) {
    if (!c || !dst) return fail(LAC_E_ARG, "bad argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(dst, c->nbits, sizeof(uint64_t) * c->B, hipMemcpyDeviceToDevice, S(stream)));
    return LAC_OK;
}

int lac_q1_k(int prec, int64_t vocab) {
    int cl = 0;
    while (((int64_t)1 << cl) < vocab) cl++;
    const int k = prec - 1 - cl;
    return k > LAC_Q1_KMAX ? LAC_Q1_KMAX : k;
}

// ---- host-side register arithmetic for predictors with their own mapping --------
// (include/lac.h "predictor-mapped coding"; no device work): lac_hc.h, shared with
// the host sanitizer build (tests/native)
int lac_hc_encode_symbol(int prec, int64_t *l, int64_t *h, int64_t lo, int64_t hi, int8_t *digits,
                         int32_t *ndigits) {
    const char *msg = "";
    const int rc = lac::hc::encode_symbol(prec, l, h, lo, hi, digits, ndigits, &msg);
    return rc ? fail(rc, "%s", msg) : LAC_OK;
}

int lac_hc_encode_flush(int prec, int64_t l, int64_t h, int8_t *digits, int32_t *ndigits) {
    const char *msg = "";
    const int rc = lac::hc::encode_flush(prec, l, h, digits, ndigits, &msg);
    return rc ? fail(rc, "%s", msg) : LAC_OK;
}

int lac_hc_decode_emit(int prec, int64_t *regs, int64_t lo, int64_t hi, int renormalise) {
    const char *msg = "";
    const int rc = lac::hc::decode_emit(prec, regs, lo, hi, renormalise, &msg);
    return rc ? fail(rc, "%s", msg) : LAC_OK;
}

int lac_profile_enable(lac_ctx *c, int on) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    c->prof = on != 0;
    return LAC_OK;
}

int lac_profile_read(lac_ctx *c, double *ms_total, int64_t *launches, int reset) {
    if (!c) return fail(LAC_E_ARG, "ctx is NULL");
    HIPCHK(hipSetDevice(c->device));
    double tot[KID_COUNT] = {0};
    int64_t cnt[KID_COUNT] = {0};
    for (auto &u : c->ev_used) {
        HIPCHK(hipEventSynchronize(u.second.second));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, u.second.first, u.second.second));
        tot[u.first] += ms;
        cnt[u.first] += 1;
    }
    for (int k = 0; k < KID_COUNT; k++) {
        if (ms_total) ms_total[k] = tot[k];
        if (launches) launches[k] = cnt[k];
    }
    if (reset) {
        c->ev_used.clear();
        c->ev_next = 0;
    }
    return LAC_OK;
}

}  // extern "C"
