// vcfc_api.cpp -- the C ABI (include/vcfc.h): contexts, device buffers and
// the host-side drivers that mirror the reference's compress() loop
// (src/compress.cpp:205-257) around the GPU encoder.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <sys/uio.h>

#include "vcfc.h"
#include "vcfc_decode_driver.h"
#include "vcfc_device.h"
#include "vcfc_ingest_driver.h"

hipError_t vcfc_sparse_plan_launch(const uint8_t *recs, const uint64_t *rec_off, uint64_t n, uint64_t data_start,
                                   uint64_t *file_off, uint8_t *prefix, uint64_t *status, hipStream_t s);
hipError_t vcfc_synth_device(uint8_t *buf, const uint64_t *line_off, uint64_t n, const uint8_t *prefix,
                             const uint64_t *prefix_off, const float *row_af, uint32_t S, int law,
                             uint64_t seed, uint64_t row_base, hipStream_t s);

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes, 1 << 20);
        want = want + want / 8;
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Pinned host memory (the ingest pipeline's staging slots).
struct HostBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        const size_t want = std::max<size_t>(std::max<size_t>(bytes, 2 * cap), 4096);   // geometric growth
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

}  // namespace

struct vcfc_timer {
    std::vector<hipEvent_t> ev;   // 6 per timed call (vcfc_encode_device)
    size_t used = 0;
};

struct vcfc_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf in, off, len, out, rec, ws, err, aux, flag, qref;
    DevBuf ing_dev[vcfc_ing::Memory::N_DEV];
    HostBuf ing_host[vcfc_ing::Memory::N_HOST];
    HostBuf dec_host[vcfc_dec::Buffers::N_HOST];
    uint64_t ingest_chunk = 0;   // 0: default (128 MiB)
    int line_index = VCFC_LINE_INDEX_HOP;
    int defer_records = VCFC_DEFER_DEFAULT;   // vcfc_ctx_set_deferred_records (on by default)
    unsigned trace = 0;          // VCFC_TRACE_* flags
};

namespace {

// Read-only mapping of an input file.
struct MappedFile {
    int fd = -1;
    const uint8_t *p = nullptr;
    uint64_t n = 0;
    int open_ro(const char *path) {
        fd = open(path, O_RDONLY);
        if (fd < 0) return VCFC_E_IO;
        struct stat st;
        if (fstat(fd, &st) != 0) return VCFC_E_IO;
        n = (uint64_t)st.st_size;
        if (n) {
            void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
            if (m == MAP_FAILED) return VCFC_E_IO;
            madvise(m, n, MADV_SEQUENTIAL);
            p = static_cast<const uint8_t *>(m);
        }
        return VCFC_OK;
    }
    ~MappedFile() {
        if (p) munmap(const_cast<uint8_t *>(p), n);
        if (fd >= 0) close(fd);
    }
};

// Metadata + header lines of a .vcfc: vcfc_dec::parse_header.
int parse_vcfc_header(const uint8_t *in, uint64_t n, uint64_t *data_off, uint64_t *sample_count) {
    return vcfc_dec::parse_header(in, n, data_off, sample_count);
}

// Record starts by hopping the LEN headers (read_compressed_line_length_headers,
// src/compress.cpp:270-331; both headers must carry extension count 3,
// src/utils.hpp:198-206).  rec[i] = offset of record i from `base`, rec[n] = end.
int index_records(const uint8_t *base, uint64_t n, std::vector<uint64_t> &rec) {
    rec.clear();
    uint64_t ip = 0;
    while (n - ip >= 8) {
        const uint8_t *h = base + ip;
        if ((h[0] >> 6) != 3 || (h[4] >> 6) != 3) return VCFC_E_FORMAT;
        const uint32_t L = ((uint32_t)(h[0] & 0x3F) << 24) | ((uint32_t)h[1] << 16) | ((uint32_t)h[2] << 8) | h[3];
        if (L < 4 || n - ip - 8 < (uint64_t)L - 4) return VCFC_E_FORMAT;
        rec.push_back(ip);
        ip += 8 + (L - 4);
    }
    rec.push_back(ip);
    return ip == n ? VCFC_OK : VCFC_E_FORMAT;
}

int write_all_at(int fd, const void *p, uint64_t len, uint64_t off) {
    const uint8_t *b = static_cast<const uint8_t *>(p);
    while (len) {
        ssize_t k = pwrite(fd, b, std::min<uint64_t>(len, 1ull << 30), (off_t)off);
        if (k <= 0) return VCFC_E_IO;
        b += k; len -= (uint64_t)k; off += (uint64_t)k;
    }
    return VCFC_OK;
}

void put_be64(uint8_t *o, uint64_t v) {
    for (int k = 0; k < 8; k++) o[k] = (uint8_t)(v >> (56 - 8 * k));
}

// The decoder's device buffers live in the context.
struct CtxDecodeBuffers : vcfc_dec::Buffers {
    vcfc_ctx *c;
    explicit CtxDecodeBuffers(vcfc_ctx *cc) : c(cc) {}
    void *get(int slot, uint64_t bytes) override {
        DevBuf *b = slot == IN ? &c->in : slot == REC ? &c->rec : slot == WS ? &c->ws : slot == OUT ? &c->out
                  : slot == LINE_OFF ? &c->off : slot == FLAG ? &c->flag
                  : slot == QREF ? &c->qref : &c->err;
        return b->ensure(bytes) == hipSuccess ? b->p : nullptr;
    }
    uint8_t *host(int slot, uint64_t bytes) override {   // pinned staging
        HostBuf &b = c->dec_host[slot];
        return b.ensure(bytes) == hipSuccess ? static_cast<uint8_t *>(b.p) : nullptr;
    }
};

// The ingest pipeline's buffers live in the context.
struct CtxIngestMemory : vcfc_ing::Memory {
    vcfc_ctx *c;
    explicit CtxIngestMemory(vcfc_ctx *cc) : c(cc) {}
    void *dev(int slot, uint64_t bytes) override {
        DevBuf &b = c->ing_dev[slot];
        return b.ensure(bytes) == hipSuccess ? b.p : nullptr;
    }
    void *host(int slot, uint64_t bytes) override {
        HostBuf &b = c->ing_host[slot];
        return b.ensure(bytes) == hipSuccess ? b.p : nullptr;
    }
};

// bytes [base, base + n) of a file
struct FdSource : vcfc_ing::Source {
    int fd;
    uint64_t n, base;
    FdSource(int f, uint64_t size, uint64_t base_off = 0) : fd(f), n(size), base(base_off) {}
    uint64_t size() const override { return n; }
    bool read(uint8_t *dst, uint64_t off, uint64_t k) override {
        off += base;
        while (k) {
            const ssize_t r = pread(fd, dst, std::min<uint64_t>(k, 1ull << 30), (off_t)off);
            if (r <= 0) return false;
            dst += r; off += (uint64_t)r; k -= (uint64_t)r;
        }
        return true;
    }
};

struct MemSource : vcfc_ing::Source {
    const uint8_t *p;
    uint64_t n;
    MemSource(const uint8_t *b, uint64_t size) : p(b), n(size) {}
    uint64_t size() const override { return n; }
    bool read(uint8_t *dst, uint64_t off, uint64_t k) override {
        memcpy(dst, p + off, k);
        return true;
    }
};

// chunk size: the context's (vcfc_ctx_set_ingest_chunk), else 128 MiB; never
// more than the input (rounded up to 4 KiB)
vcfc_ing::Config ingest_config(const vcfc_ctx *c, uint64_t n) {
    vcfc_ing::Config cfg;
    const uint64_t want = c->ingest_chunk ? c->ingest_chunk : (128ull << 20);
    cfg.chunk = std::min<uint64_t>(want, std::max<uint64_t>((n + 4095) & ~4095ull, 4096));
    cfg.trace = (c->trace & VCFC_TRACE_INGEST) != 0;
    cfg.defer_records = c->defer_records != 0;
    return cfg;
}

}  // namespace

extern "C" {

const char *vcfc_version(void) { return "vcfc-mi355x 0.1 (gfx950)"; }

const char *vcfc_strerror(int s) {
    switch (s) {
    case VCFC_OK: return "ok";
    case VCFC_E_LT8COLS: return "VCF data line did not contain at least 8 terms";
    case VCFC_E_8COLS: return "VCF data line has exactly 8 terms (reference aborts: std::length_error)";
    case VCFC_E_HEADER: return "VCF Header did not have enough columns";
    case VCFC_E_NOSPACE: return "output buffer too small";
    case VCFC_E_ARG: return "invalid argument";
    case VCFC_E_HIP: return "HIP runtime error (is a gfx950 GPU visible?)";
    case VCFC_E_IO: return "file I/O error";
    case VCFC_E_FORMAT: return "malformed .vcfc input";
    case VCFC_E_TOOLONG: return "VCF data line too long (its record could pass the 30-bit length header)";
    default: return "unknown status";
    }
}

int vcfc_ctx_create(int device, vcfc_ctx **out) {
    if (!out) return VCFC_E_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || device >= n) return VCFC_E_HIP;
    if (hipSetDevice(device) != hipSuccess) return VCFC_E_HIP;
    vcfc_ctx *c = new vcfc_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return VCFC_E_HIP;
    }
    *out = c;
    return VCFC_OK;
}

void vcfc_ctx_destroy(vcfc_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    c->in.release(); c->off.release(); c->len.release(); c->out.release();
    c->rec.release(); c->ws.release(); c->err.release(); c->aux.release();
    c->flag.release(); c->qref.release();
    for (auto &b : c->ing_dev) b.release();
    for (auto &b : c->ing_host) b.release();
    for (auto &b : c->dec_host) b.release();
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int vcfc_ctx_set_ingest_chunk(vcfc_ctx *c, uint64_t chunk_bytes) {
    if (!c || (chunk_bytes && (chunk_bytes < 4096 || chunk_bytes > (3ull << 30)))) return VCFC_E_ARG;
    c->ingest_chunk = chunk_bytes;
    return VCFC_OK;
}

int vcfc_ctx_set_line_index(vcfc_ctx *c, int mode) {
    if (!c || (mode != VCFC_LINE_INDEX_HOP && mode != VCFC_LINE_INDEX_SCAN)) return VCFC_E_ARG;
    c->line_index = mode;
    return VCFC_OK;
}

int vcfc_ctx_set_deferred_records(vcfc_ctx *c, int on) {
    if (!c || (on != 0 && on != 1)) return VCFC_E_ARG;
    c->defer_records = on;
    return VCFC_OK;
}

int vcfc_ctx_set_trace(vcfc_ctx *c, unsigned flags) {
    if (!c || (flags & ~(VCFC_TRACE_INGEST | VCFC_TRACE_DEVICE | VCFC_TRACE_SPARSE_QUERY))) return VCFC_E_ARG;
    c->trace = flags;
    return VCFC_OK;
}

uint64_t vcfc_encode_bound(uint64_t n_rows, uint64_t total_line_bytes) {
    return vcfc_record_bound(n_rows, total_line_bytes);
}

uint64_t vcfc_encode_workspace_size(uint64_t n_rows, uint64_t total_line_bytes) {
    return vcfc_encode_workspace_layout(n_rows, total_line_bytes).total;
}

static int encode_rows_device_impl(const uint8_t *d_buf, const uint64_t *d_line_off, const uint32_t *d_line_len,
                                   uint64_t n, uint64_t total_line_bytes, uint8_t *d_out, uint64_t out_cap,
                                   uint64_t *d_rec_off, void *d_ws, uint64_t ws_bytes, uint64_t *d_err, void *stream,
                                   hipEvent_t *ev) {
    if ((n && (!d_buf || !d_line_off || !d_line_len || !d_out)) || !d_rec_off || !d_err || (n && !d_ws))
        return VCFC_E_ARG;
    const VcfcWorkspaceLayout L = vcfc_encode_workspace_layout(n, total_line_bytes);
    if (ws_bytes < L.total) return VCFC_E_NOSPACE;
    uint8_t *ws = static_cast<uint8_t *>(d_ws);
    VcfcEncodeArgs a;
    a.buf = d_buf;
    a.line_off = d_line_off;
    a.line_len = d_line_len;
    a.n = n;
    a.line_bytes_hint = total_line_bytes;
    a.out = d_out;
    a.out_cap = out_cap;
    a.rec_off = d_rec_off;
    vcfc_encode_args_workspace(a, ws, L);
    a.err = d_err;
    return vcfc_encode_device(a, static_cast<hipStream_t>(stream), ev) == hipSuccess ? VCFC_OK : VCFC_E_HIP;
}

int vcfc_encode_rows_device(const uint8_t *d_buf, const uint64_t *d_line_off, const uint32_t *d_line_len,
                            uint64_t n, uint64_t total_line_bytes, uint8_t *d_out, uint64_t out_cap,
                            uint64_t *d_rec_off, void *d_ws, uint64_t ws_bytes, uint64_t *d_err, void *stream) {
    return encode_rows_device_impl(d_buf, d_line_off, d_line_len, n, total_line_bytes, d_out, out_cap, d_rec_off,
                                   d_ws, ws_bytes, d_err, stream, nullptr);
}

int vcfc_encode_deferred_rows(const void *d_ws, uint64_t n, uint64_t total_line_bytes, void *stream,
                              uint64_t *rows) {
    if (!rows || (n && !d_ws)) return VCFC_E_ARG;
    *rows = 0;
    if (n == 0) return VCFC_OK;
    const VcfcWorkspaceLayout L = vcfc_encode_workspace_layout(n, total_line_bytes);
    uint32_t v = 0, fb = 0;   // deferred by k_encode_var, of which taken by the general path after all
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint8_t *ws = static_cast<const uint8_t *>(d_ws);
    if (hipMemcpyAsync(&v, ws + vcfc_defer_count_offset(L), 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(&fb, ws + vcfc_defer_fallback_offset(L), 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return VCFC_E_HIP;
    *rows = v - fb;
    return VCFC_OK;
}

int vcfc_timer_create(vcfc_timer **t) {
    if (!t) return VCFC_E_ARG;
    *t = new vcfc_timer();
    return VCFC_OK;
}

void vcfc_timer_destroy(vcfc_timer *t) {
    if (!t) return;
    for (auto &e : t->ev) (void)hipEventDestroy(e);
    delete t;
}

int vcfc_encode_rows_device_timed(const uint8_t *d_buf, const uint64_t *d_line_off, const uint32_t *d_line_len,
                                  uint64_t n, uint64_t total_line_bytes, uint8_t *d_out, uint64_t out_cap,
                                  uint64_t *d_rec_off, void *d_ws, uint64_t ws_bytes, uint64_t *d_err, void *stream,
                                  vcfc_timer *t) {
    if (!t) return VCFC_E_ARG;
    const size_t base = 6 * t->used;
    while (t->ev.size() < base + 6) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return VCFC_E_HIP;
        t->ev.push_back(e);
    }
    int st = encode_rows_device_impl(d_buf, d_line_off, d_line_len, n, total_line_bytes, d_out, out_cap, d_rec_off,
                                     d_ws, ws_bytes, d_err, stream, t->ev.data() + base);
    if (st == VCFC_OK) t->used++;
    return st;
}

int vcfc_timer_read(vcfc_timer *t, double ms[4], uint64_t *calls) {
    if (!t || !ms) return VCFC_E_ARG;
    for (int k = 0; k < 4; k++) ms[k] = 0;
    for (size_t i = 0; i < t->used; i++) {
        hipEvent_t *e = t->ev.data() + 6 * i;
        if (hipEventSynchronize(e[5]) != hipSuccess) return VCFC_E_HIP;
        for (int k = 0; k < 5; k++) {
            float f = 0;
            if (hipEventElapsedTime(&f, e[k], e[k + 1]) != hipSuccess) return VCFC_E_HIP;
            ms[k == 4 ? 1 : k] += f;   // k_encode_defer's deferred records count as k_encode
        }
    }
    if (calls) *calls = t->used;
    t->used = 0;
    return VCFC_OK;
}

int vcfc_synth_rows_device_at(uint8_t *d_buf, const uint64_t *d_line_off, uint64_t n, const uint8_t *d_prefix,
                              const uint64_t *d_prefix_off, const float *d_row_af, uint32_t samples, int law,
                              uint64_t seed, uint64_t row_base, void *stream) {
    if (n && (!d_buf || !d_line_off || !d_prefix || !d_prefix_off)) return VCFC_E_ARG;
    if (law < 0 || law > 3 || (law >= 2 && n && !d_row_af)) return VCFC_E_ARG;
    return vcfc_synth_device(d_buf, d_line_off, n, d_prefix, d_prefix_off, d_row_af, samples, law, seed, row_base,
                             static_cast<hipStream_t>(stream)) == hipSuccess
               ? VCFC_OK
               : VCFC_E_HIP;
}

int vcfc_synth_rows_device(uint8_t *d_buf, const uint64_t *d_line_off, uint64_t n, const uint8_t *d_prefix,
                           const uint64_t *d_prefix_off, const float *d_row_af, uint32_t samples, int law,
                           uint64_t seed, void *stream) {
    return vcfc_synth_rows_device_at(d_buf, d_line_off, n, d_prefix, d_prefix_off, d_row_af, samples, law, seed, 0,
                                     stream);
}

// Host batch: copy in, encode, copy out.  Synchronous on the context stream.
int vcfc_encode_rows(vcfc_ctx *c, const uint8_t *buf, uint64_t buf_bytes, const uint64_t *line_off,
                     const uint32_t *line_len, uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *rec_off,
                     int64_t *err_row) {
    if (!c || !rec_off || (n && (!buf || !line_off || !line_len || !out))) return VCFC_E_ARG;
    if (err_row) *err_row = -1;
    if (hipSetDevice(c->device) != hipSuccess) return VCFC_E_HIP;
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (line_off[i] + line_len[i] > buf_bytes) return VCFC_E_ARG;
        total += line_len[i];
    }
    const uint64_t bound = vcfc_encode_bound(n, total);
    const uint64_t wsz = vcfc_encode_workspace_size(n, total);
    if (c->in.ensure(buf_bytes + 64) || c->off.ensure(8 * n + 8) || c->len.ensure(4 * n + 8) ||
        c->out.ensure(bound) || c->rec.ensure(8 * (n + 1)) || c->ws.ensure(wsz) || c->err.ensure(8))
        return VCFC_E_HIP;
    hipStream_t s = c->stream;
    if (hipMemcpyAsync(c->in.p, buf, buf_bytes, hipMemcpyHostToDevice, s) ||
        hipMemcpyAsync(c->off.p, line_off, 8 * n, hipMemcpyHostToDevice, s) ||
        hipMemcpyAsync(c->len.p, line_len, 4 * n, hipMemcpyHostToDevice, s))
        return VCFC_E_HIP;
    int st = vcfc_encode_rows_device(static_cast<uint8_t *>(c->in.p), static_cast<uint64_t *>(c->off.p),
                                     static_cast<uint32_t *>(c->len.p), n, total, static_cast<uint8_t *>(c->out.p),
                                     c->out.cap, static_cast<uint64_t *>(c->rec.p), c->ws.p, c->ws.cap,
                                     static_cast<uint64_t *>(c->err.p), s);
    if (st != VCFC_OK) return st;
    uint64_t errw = 0;
    if (hipMemcpyAsync(rec_off, c->rec.p, 8 * (n + 1), hipMemcpyDeviceToHost, s) ||
        hipMemcpyAsync(&errw, c->err.p, 8, hipMemcpyDeviceToHost, s) || hipStreamSynchronize(s))
        return VCFC_E_HIP;
    uint64_t upto = n, status = VCFC_OK;
    if (errw != VCFCD_NO_ERROR) {
        upto = errw >> 8;
        status = errw & 0xFF;
        if (err_row) *err_row = (int64_t)upto;
    }
    const uint64_t bytes = rec_off[upto];
    if (bytes > out_cap) return VCFC_E_NOSPACE;
    if (bytes && (hipMemcpyAsync(out, c->out.p, bytes, hipMemcpyDeviceToHost, s) || hipStreamSynchronize(s)))
        return VCFC_E_HIP;
    return (int)status;
}

int vcfc_compress_data_line(vcfc_ctx *c, const char *line, uint64_t len, int add_newline, uint8_t *out,
                            uint64_t out_cap, uint64_t *out_len) {
    if (!c || !line || !out || !out_len || len > 0xFFFFFFFFull) return VCFC_E_ARG;
    const uint64_t off = 0;
    const uint32_t l32 = (uint32_t)len;
    uint64_t ro[2] = {0, 0};
    std::vector<uint8_t> tmp(vcfc_encode_bound(1, len) + 16);
    int64_t er = -1;
    int st = vcfc_encode_rows(c, reinterpret_cast<const uint8_t *>(line), len, &off, &l32, 1, tmp.data(),
                              tmp.size(), ro, &er);
    if (st != VCFC_OK) return st;
    uint64_t n = ro[1];
    if (!add_newline) n -= 1;  // records always end in '\n' (compress.cpp:188-190)
    if (n > out_cap) return VCFC_E_NOSPACE;
    if (!add_newline) {
        // LEN counts the record without the newline
        const uint32_t L = (uint32_t)(n - 4);
        tmp[0] = (uint8_t)(((L >> 24) & 0xFF) | 0xC0);
        tmp[1] = (uint8_t)((L >> 16) & 0xFF);
        tmp[2] = (uint8_t)((L >> 8) & 0xFF);
        tmp[3] = (uint8_t)(L & 0xFF);
    }
    memcpy(out, tmp.data(), n);
    *out_len = n;
    return VCFC_OK;
}

uint64_t vcfc_sparse_offset(uint64_t pos) { return (300000000ull + pos) * (4ull * 4096ull); }

int vcfc_sparse_plan_device(const uint8_t *d_recs, const uint64_t *d_rec_off, uint64_t n, uint64_t data_start,
                            uint64_t *d_file_off, uint8_t *d_prefix16, uint64_t *d_status, void *stream) {
    if ((n && (!d_recs || !d_rec_off || !d_file_off || !d_prefix16)) || !d_status) return VCFC_E_ARG;
    return vcfc_sparse_plan_launch(d_recs, d_rec_off, n, data_start, d_file_off, d_prefix16, d_status,
                                   static_cast<hipStream_t>(stream)) == hipSuccess
               ? VCFC_OK
               : VCFC_E_HIP;
}

// sparsify_file (reference src/sparse.cpp:290-580).  The GPU plans offsets
// and prefixes; the host writes one pwritev per record (the reference writes
// one byte per syscall) or, if the plan flags overlapping/out-of-order
// records, replays the reference's write sequence so later writes win as
// they do there.
namespace {

// Plan records [a, b) of the index on the GPU (k_sparse_plan): file offsets,
// 16-byte prefixes; status[0] = ~0 or (first unparsable record, local to a)
// << 8 | code, status[1] = 1 if adjacent records overlap or are out of order.
int sparse_plan_range(vcfc_ctx *c, const uint8_t *recs, const std::vector<uint64_t> &rec, uint64_t a, uint64_t b,
                      uint64_t data_start, std::vector<uint64_t> &file_off, std::vector<uint8_t> &prefix,
                      uint64_t status[2]) {
    const uint64_t n = b - a;
    file_off.assign(n, 0);
    prefix.assign(16 * n, 0);
    status[0] = ~0ull;
    status[1] = 0;
    if (!n) return VCFC_OK;
    const uint64_t base = rec[a], span = rec[b] - base;
    std::vector<uint64_t> ro(n + 1);
    for (uint64_t i = 0; i <= n; i++) ro[i] = rec[a + i] - base;
    if (c->in.ensure(span + 64) || c->rec.ensure(8 * (n + 1)) || c->out.ensure(16 * n) || c->off.ensure(8 * n) ||
        c->err.ensure(16))
        return VCFC_E_HIP;
    hipStream_t s = c->stream;
    if (hipMemcpyAsync(c->in.p, recs + base, span, hipMemcpyHostToDevice, s) ||
        hipMemcpyAsync(c->rec.p, ro.data(), 8 * (n + 1), hipMemcpyHostToDevice, s))
        return VCFC_E_HIP;
    if (vcfc_sparse_plan_launch(static_cast<uint8_t *>(c->in.p), static_cast<uint64_t *>(c->rec.p), n, data_start,
                                static_cast<uint64_t *>(c->off.p), static_cast<uint8_t *>(c->out.p),
                                static_cast<uint64_t *>(c->err.p), s) != hipSuccess)
        return VCFC_E_HIP;
    if (hipMemcpyAsync(file_off.data(), c->off.p, 8 * n, hipMemcpyDeviceToHost, s) ||
        hipMemcpyAsync(prefix.data(), c->out.p, 16 * n, hipMemcpyDeviceToHost, s) ||
        hipMemcpyAsync(status, c->err.p, 16, hipMemcpyDeviceToHost, s) || hipStreamSynchronize(s))
        return VCFC_E_HIP;
    return VCFC_OK;
}

// Write records g0 .. g0 + cnt - 1 (global indices; file_off / prefix point at
// record g0's plan) with one pwritev each; record 0 also fills the
// first-offset slot (host byte order, sparse.cpp:495-511).  replay (g0 == 0
// only): the reference's exact write sequence -- a record's dist_to_next goes
// out as 0 and the next record's step patches it (sparse.cpp:529-553) -- so
// later writes win where records overlap.
int sparse_write_range(int fd, const uint8_t *recs, const std::vector<uint64_t> &rec, uint64_t g0, uint64_t cnt,
                       const uint64_t *file_off, const uint8_t *prefix, uint64_t data_start, bool replay) {
    int w = VCFC_OK;
    for (uint64_t i = 0; i < cnt && !w; i++) {
        const uint64_t g = g0 + i;
        uint8_t pfx[16];
        memcpy(pfx, prefix + 16 * i, 16);
        if (g == 0) {
            const uint64_t voff = file_off[i] - data_start;
            w = write_all_at(fd, &voff, 8, data_start - 8);
        } else if (replay) {
            uint8_t d[8];
            put_be64(d, file_off[i] - file_off[i - 1]);
            w = write_all_at(fd, d, 8, file_off[i - 1] + 8);
        }
        if (w) break;
        if (replay) memset(pfx + 8, 0, 8);
        struct iovec iov[2] = {{pfx, 16}, {const_cast<uint8_t *>(recs + rec[g]), (size_t)(rec[g + 1] - rec[g])}};
        const uint64_t want = 16 + rec[g + 1] - rec[g];
        ssize_t k = pwritev(fd, iov, 2, (off_t)file_off[i]);
        if (k != (ssize_t)want) {
            // short write: finish the record plainly
            std::vector<uint8_t> tmp(want);
            memcpy(tmp.data(), pfx, 16);
            memcpy(tmp.data() + 16, recs + rec[g], want - 16);
            w = write_all_at(fd, tmp.data(), want, file_off[i]);
        }
    }
    return w;
}

// The .vcfc mapped, its header parsed and its records indexed.
struct SparseInput {
    MappedFile f;
    uint64_t data_in = 0, n = 0, data_start = 0;
    const uint8_t *recs = nullptr;
    std::vector<uint64_t> rec;
    int ist = VCFC_OK;   // index_records status (an error after the good prefix)
    int open(const char *path) {
        int st = f.open_ro(path);
        if (st) return st;
        if ((st = parse_vcfc_header(f.p, f.n, &data_in, nullptr))) return st;
        recs = f.p + data_in;
        ist = index_records(recs, f.n - data_in, rec);
        n = rec.size() - 1;
        data_start = data_in + 8;   // header lines + 8-byte slot
        return VCFC_OK;
    }
};

}  // namespace

int vcfc_sparsify_file(vcfc_ctx *c, const char *in_path, const char *out_path) {
    if (!c || !in_path || !out_path) return VCFC_E_ARG;
    if (hipSetDevice(c->device) != hipSuccess) return VCFC_E_HIP;
    SparseInput in;
    int st = in.open(in_path);
    if (st) return st;
    const uint64_t n = in.n;
    std::vector<uint64_t> file_off;
    std::vector<uint8_t> prefix;
    uint64_t status[2];
    if ((st = sparse_plan_range(c, in.recs, in.rec, 0, n, in.data_start, file_off, prefix, status))) return st;
    uint64_t upto = n;   // records before the first unparsable one are written
    if (status[0] != ~0ull && n) upto = status[0] >> 8;
    int fd = open(out_path, O_CREAT | O_TRUNC | O_RDWR, 0600);
    if (fd < 0) return VCFC_E_IO;
    int w = write_all_at(fd, in.f.p, in.data_in, 0);
    const uint8_t zero8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (!w) w = write_all_at(fd, zero8, 8, in.data_in);
    if (!w)
        w = sparse_write_range(fd, in.recs, in.rec, 0, upto, file_off.data(), prefix.data(), in.data_start,
                               status[1] != 0);
    close(fd);
    if (w) return w;
    if (upto < n) return VCFC_E_FORMAT;
    return in.ist;
}

int vcfc_sparsify_shard(vcfc_ctx *c, const char *in_path, const char *out_path, int rank, int world,
                        uint64_t info[4]) {
    if (!c || !in_path || !info || world < 1 || rank < 0 || rank >= world) return VCFC_E_ARG;
    if (hipSetDevice(c->device) != hipSuccess) return VCFC_E_HIP;
    SparseInput in;
    int st = in.open(in_path);
    if (st) return st;
    const uint64_t n = in.n;
    const uint64_t lo = (uint64_t)((unsigned __int128)n * (unsigned)rank / (unsigned)world);
    const uint64_t hi = (uint64_t)((unsigned __int128)n * (unsigned)(rank + 1) / (unsigned)world);
    const uint64_t a = lo ? lo - 1 : 0, b = hi < n ? hi + 1 : n;   // one halo record each side
    std::vector<uint64_t> file_off;
    std::vector<uint8_t> prefix;
    uint64_t status[2] = {~0ull, 0};
    if (hi > lo && (st = sparse_plan_range(c, in.recs, in.rec, a, b, in.data_start, file_off, prefix, status)))
        return st;
    info[0] = lo;
    info[1] = hi;
    info[2] = status[0] != ~0ull ? a + (status[0] >> 8) : (in.ist ? n : ~0ull);
    info[3] = status[1];
    if (!out_path) return VCFC_OK;
    if (info[2] != ~0ull || info[3]) return VCFC_E_ARG;
    int fd = open(out_path, O_CREAT | O_WRONLY, 0600);
    if (fd < 0) return VCFC_E_IO;
    int w = VCFC_OK;
    if (rank == 0) {
        w = write_all_at(fd, in.f.p, in.data_in, 0);
        const uint8_t zero8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (!w && n == 0) w = write_all_at(fd, zero8, 8, in.data_in);   // else record 0's owner fills it
    }
    if (!w && hi > lo)
        w = sparse_write_range(fd, in.recs, in.rec, lo, hi - lo, file_off.data() + (lo - a),
                               prefix.data() + 16 * (lo - a), in.data_start, false);
    close(fd);
    return w;
}

uint64_t vcfc_compress_bound(uint64_t in_bytes) { return in_bytes + in_bytes / 2 + 64; }

// compress() (reference src/compress.cpp:205-257) through the pipelined
// ingest (csrc/vcfc_ingest_driver.h: reader threads -> GPU line index +
// encode -> writer thread).
int vcfc_compress_buffer(vcfc_ctx *c, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap,
                         uint64_t *out_len, int64_t *err_line) {
    if (!c || (!in && n) || !out || !out_len) return VCFC_E_ARG;
    if (err_line) *err_line = -1;
    *out_len = 0;
    if (hipSetDevice(c->device) != hipSuccess) return VCFC_E_HIP;
    uint64_t o = 0;
    bool full = false;
    auto sink = [&](const uint8_t *p, uint64_t k) {
        if (o + k > out_cap) { full = true; return false; }
        memcpy(out + o, p, k);
        o += k;
        return true;
    };
    MemSource src(in, n);
    CtxIngestMemory M(c);
    const vcfc_ing::Config cfg = ingest_config(c, n);
    const int st = vcfc_ing::compress_stream(src, sink, M, c->stream, cfg, err_line);
    *out_len = o;
    if (full) return VCFC_E_NOSPACE;
    return st;
}

// compress() over VCF file bytes resident in device memory: line index +
// encoder on the GPU over the whole input at once (or chunks of the context's
// ingest chunk when one is set), output left in device memory
// (vcfc_ing::compress_device).
int vcfc_compress_device(vcfc_ctx *c, const uint8_t *d_in, uint64_t n, uint8_t *d_out, uint64_t out_cap,
                         uint64_t *out_len, int64_t *err_line) {
    if (!c || (!d_in && n) || !d_out || !out_len) return VCFC_E_ARG;
    if (err_line) *err_line = -1;
    *out_len = 0;
    if (hipSetDevice(c->device) != hipSuccess) return VCFC_E_HIP;
    CtxIngestMemory M(c);
    vcfc_ing::Config cfg;
    cfg.max_chunk = 1ull << 40;   // (line lengths are 32-bit; the index's positions 64-bit)
    const uint64_t want = c->ingest_chunk ? c->ingest_chunk : cfg.max_chunk;
    cfg.chunk = std::min<uint64_t>(want, std::max<uint64_t>((n + 4095) & ~4095ull, 4096));
    cfg.hop_index = c->line_index == VCFC_LINE_INDEX_HOP;
    cfg.defer_records = c->defer_records != 0;
    cfg.trace = (c->trace & VCFC_TRACE_DEVICE) != 0;
    return vcfc_ing::compress_device(d_in, n, d_out, out_cap, out_len, M, c->stream, cfg, err_line);
}

int vcfc_compress_file(vcfc_ctx *c, const char *in_path, const char *out_path, int64_t *err_line) {
    if (!c || !in_path || !out_path) return VCFC_E_ARG;
    if (err_line) *err_line = -1;
    if (hipSetDevice(c->device) != hipSuccess) return VCFC_E_HIP;
    int fd = open(in_path, O_RDONLY);
    if (fd < 0) return VCFC_E_IO;
    struct stat st;
    if (fstat(fd, &st) != 0) { close(fd); return VCFC_E_IO; }
    const uint64_t n = (uint64_t)st.st_size;
    posix_fadvise(fd, 0, 0, POSIX_FADV_SEQUENTIAL);
    // the reference opens (truncates) the output before reading the input
    int ofd = open(out_path, O_CREAT | O_TRUNC | O_WRONLY, 0644);
    if (ofd < 0) { close(fd); return VCFC_E_IO; }
    auto sink = [&](const uint8_t *p, uint64_t k) {
        while (k) {
            const ssize_t w = write(ofd, p, std::min<uint64_t>(k, 1ull << 30));
            if (w <= 0) return false;
            p += w;
            k -= (uint64_t)w;
        }
        return true;
    };
    FdSource src(fd, n);
    CtxIngestMemory M(c);
    const vcfc_ing::Config cfg = ingest_config(c, n);
    int s = vcfc_ing::compress_stream(src, sink, M, c->stream, cfg, err_line);
    close(fd);
    if (close(ofd) != 0 && s == VCFC_OK) s = VCFC_E_IO;
    return s;
}

// One rank's share of a sharded compress (SURVEY §8 e): the line-aligned byte
// range [off, off + len) of in_path through the same pipeline, its output
// written to out_fd from out_off on (pwrite; the caller places it).
int vcfc_compress_range(vcfc_ctx *c, const char *in_path, uint64_t off, uint64_t len, int out_fd, uint64_t out_off,
                        uint64_t *out_bytes, int64_t *err_line, uint64_t *lines) {
    if (!c || !in_path || out_fd < 0 || !out_bytes) return VCFC_E_ARG;
    *out_bytes = 0;
    if (err_line) *err_line = -1;
    if (lines) *lines = 0;
    if (hipSetDevice(c->device) != hipSuccess) return VCFC_E_HIP;
    int fd = open(in_path, O_RDONLY);
    if (fd < 0) return VCFC_E_IO;
    struct stat st;
    if (fstat(fd, &st) != 0 || off > (uint64_t)st.st_size || len > (uint64_t)st.st_size - off) {
        close(fd);
        return VCFC_E_ARG;
    }
    posix_fadvise(fd, (off_t)off, (off_t)len, POSIX_FADV_SEQUENTIAL);
    uint64_t o = 0;
    auto sink = [&](const uint8_t *p, uint64_t k) {
        if (write_all_at(out_fd, p, k, out_off + o)) return false;
        o += k;
        return true;
    };
    FdSource src(fd, len, off);
    CtxIngestMemory M(c);
    const vcfc_ing::Config cfg = ingest_config(c, len);
    const int s = vcfc_ing::compress_stream(src, sink, M, c->stream, cfg, err_line, lines);
    close(fd);
    *out_bytes = o;
    return s;
}

struct vcfc_held : vcfc_ing::Held {};

int vcfc_compress_range_held(vcfc_ctx *c, const char *in_path, uint64_t off, uint64_t len, uint64_t mem_bound,
                             const char *spill_dir, vcfc_held **held, uint64_t *out_bytes, int64_t *err_line,
                             uint64_t *lines) {
    if (!c || !in_path || !held || !out_bytes) return VCFC_E_ARG;
    *held = nullptr;
    *out_bytes = 0;
    if (err_line) *err_line = -1;
    if (lines) *lines = 0;
    if (hipSetDevice(c->device) != hipSuccess) return VCFC_E_HIP;
    int fd = open(in_path, O_RDONLY);
    if (fd < 0) return VCFC_E_IO;
    struct stat st;
    if (fstat(fd, &st) != 0 || off > (uint64_t)st.st_size || len > (uint64_t)st.st_size - off) {
        close(fd);
        return VCFC_E_ARG;
    }
    posix_fadvise(fd, (off_t)off, (off_t)len, POSIX_FADV_SEQUENTIAL);
    vcfc_held *h = new (std::nothrow) vcfc_held;
    if (!h) { close(fd); return VCFC_E_IO; }
    h->mem_bound = mem_bound;
    if (spill_dir) h->spill_dir = spill_dir;
    auto sink = [&](const uint8_t *p, uint64_t k) { return h->append(p, k); };
    FdSource src(fd, len, off);
    CtxIngestMemory M(c);
    const vcfc_ing::Config cfg = ingest_config(c, len);
    const int s = vcfc_ing::compress_stream(src, sink, M, c->stream, cfg, err_line, lines);
    close(fd);
    *held = h;
    *out_bytes = h->bytes();
    return s;
}

int vcfc_held_place(const vcfc_held *h, int out_fd, uint64_t out_off) {
    if (!h || out_fd < 0) return VCFC_E_ARG;
    return h->place(out_fd, out_off) ? VCFC_OK : VCFC_E_IO;
}

void vcfc_held_sizes(const vcfc_held *h, uint64_t *mem_bytes, uint64_t *spill_bytes) {
    if (mem_bytes) *mem_bytes = h ? h->mem : 0;
    if (spill_bytes) *spill_bytes = h ? h->spilled : 0;
}

void vcfc_held_free(vcfc_held *h) { delete h; }

// ---- decoder: decompress2_fd, reference
// src/compress.cpp:1214-1257 ------------------------------------------------

int vcfc_decompress_buffer(vcfc_ctx *c, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap,
                           uint64_t *out_len) {
    if (!c || (!in && n) || (!out && out_cap) || !out_len) return VCFC_E_ARG;
    *out_len = 0;
    if (hipSetDevice(c->device) != hipSuccess) return VCFC_E_HIP;
    uint64_t data_off = 0, S = 0;
    int st = parse_vcfc_header(in, n, &data_off, &S);
    if (st) return st;   // the reference writes nothing before its header check passes
    uint64_t o = 0;
    bool fits = true;
    auto sink = [&](const uint8_t *p, uint64_t k) {
        if (fits && o + k <= out_cap) memcpy(out + o, p, k);
        else fits = false;
        o += k;
        return true;
    };
    sink(in, data_off);
    CtxDecodeBuffers B(c);
    st = vcfc_dec::decode_section(in + data_off, n - data_off, S, B, c->stream, sink);
    *out_len = o;
    if (!fits) return VCFC_E_NOSPACE;
    return st;
}

int vcfc_decompress_file(vcfc_ctx *c, const char *in_path, const char *out_path) {
    if (!c || !in_path || !out_path) return VCFC_E_ARG;
    if (hipSetDevice(c->device) != hipSuccess) return VCFC_E_HIP;
    MappedFile f;
    int st = f.open_ro(in_path);
    if (st) return st;
    // the reference opens (truncates) the output before reading the headers
    int fd = open(out_path, O_CREAT | O_TRUNC | O_WRONLY, 0644);
    if (fd < 0) return VCFC_E_IO;
    uint64_t data_off = 0, S = 0;
    st = parse_vcfc_header(f.p, f.n, &data_off, &S);
    uint64_t o = 0;
    auto sink = [&](const uint8_t *p, uint64_t k) {
        if (write_all_at(fd, p, k, o)) return false;
        o += k;
        return true;
    };
    if (!st && !sink(f.p, data_off)) st = VCFC_E_IO;
    if (!st) {
        CtxDecodeBuffers B(c);
        st = vcfc_dec::decode_section(f.p + data_off, f.n - data_off, S, B, c->stream, sink);
    }
    close(fd);
    return st;
}

// ---- range query: query_compressed_file, reference
// src/main.cpp:3777-3929 ----------------------------------------------------

// parse_coordinate_string (src/main.cpp:3993-4026) with str_to_uint64
// (src/utils.cpp:152-165: strtoul over the whole string; "" parses as 0)
static bool str_to_u64(const char *s, uint64_t n, uint64_t *out) {
    if (n == 0) { *out = 0; return true; }
    uint64_t i = 0;
    while (i < n && (s[i] == ' ' || (s[i] >= '\t' && s[i] <= '\r'))) i++;
    bool neg = false;
    if (i < n && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; i++; }
    if (i >= n || s[i] < '0' || s[i] > '9') return false;
    uint64_t v = 0;
    bool ovf = false;
    for (; i < n && s[i] >= '0' && s[i] <= '9'; i++) {
        const uint64_t d = (uint64_t)(s[i] - '0');
        ovf = ovf || v > (UINT64_MAX - d) / 10;
        v = v * 10 + d;
    }
    if (i != n) return false;
    *out = ovf ? UINT64_MAX : (neg ? 0 - v : v);
    return true;
}

int vcfc_parse_query(const char *q, uint64_t q_len, uint64_t *ref_len, int *has_range, uint64_t *start,
                     uint64_t *end) {
    if ((!q && q_len) || !ref_len || !has_range || !start || !end) return VCFC_E_ARG;
    const char *colon = q_len ? static_cast<const char *>(memchr(q, ':', q_len)) : nullptr;
    if (!colon) {
        *ref_len = q_len; *has_range = 0; *start = *end = 0;
        return 0;
    }
    const uint64_t ci = (uint64_t)(colon - q);
    const char *dash = static_cast<const char *>(memchr(q + ci + 1, '-', q_len - ci - 1));
    if (!dash) return 1;
    const uint64_t di = (uint64_t)(dash - q);
    if (!str_to_u64(q + ci + 1, di - ci - 1, start)) return 2;
    if (!str_to_u64(q + di + 1, q_len - di - 1, end)) return 3;
    *ref_len = ci;
    *has_range = 1;
    return 0;
}

int vcfc_query_buffer(vcfc_ctx *c, const uint8_t *in, uint64_t n, const char *ref, uint64_t ref_len, int has_range,
                      uint64_t start, uint64_t end, uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if (!c || (!in && n) || (!ref && ref_len) || (!out && out_cap) || !out_len) return VCFC_E_ARG;
    *out_len = 0;
    if (hipSetDevice(c->device) != hipSuccess) return VCFC_E_HIP;
    uint64_t data_off = 0, S = 0;
    int st = parse_vcfc_header(in, n, &data_off, &S);
    if (st) return st;
    uint64_t o = 0;
    bool fits = true;
    auto sink = [&](const uint8_t *p, uint64_t k) {
        if (fits && o + k <= out_cap) memcpy(out + o, p, k);
        else fits = false;
        o += k;
        return true;
    };
    CtxDecodeBuffers B(c);
    st = vcfc_dec::query_section(in + data_off, n - data_off, S, reinterpret_cast<const uint8_t *>(ref), ref_len,
                                 has_range, start, end, B, c->stream, sink);
    *out_len = o;
    if (!fits) return VCFC_E_NOSPACE;
    return st;
}

int vcfc_query_file(vcfc_ctx *c, const char *in_path, const char *ref, uint64_t ref_len, int has_range,
                    uint64_t start, uint64_t end, int out_fd) {
    if (!c || !in_path || (!ref && ref_len) || out_fd < 0) return VCFC_E_ARG;
    if (hipSetDevice(c->device) != hipSuccess) return VCFC_E_HIP;
    MappedFile f;
    int st = f.open_ro(in_path);
    if (st) return st;
    uint64_t data_off = 0, S = 0;
    if ((st = parse_vcfc_header(f.p, f.n, &data_off, &S))) return st;
    auto sink = [&](const uint8_t *p, uint64_t k) {
        while (k) {
            const ssize_t w = write(out_fd, p, std::min<uint64_t>(k, 1ull << 30));
            if (w <= 0) return false;
            p += w;
            k -= (uint64_t)w;
        }
        return true;
    };
    CtxDecodeBuffers B(c);
    return vcfc_dec::query_section(f.p + data_off, f.n - data_off, S, reinterpret_cast<const uint8_t *>(ref), ref_len,
                                   has_range, start, end, B, c->stream, sink);
}

// ---- sparse-file query: query_sparse_file_fd, reference
// src/main.cpp:235-582 ------------------------------------------------------
int vcfc_sparse_query_file(vcfc_ctx *c, const char *in_path, const char *ref, uint64_t ref_len, int has_range,
                           uint64_t start, uint64_t end, int out_fd) {
    if (!c || !in_path || (!ref && ref_len) || out_fd < 0) return VCFC_E_ARG;
    if (hipSetDevice(c->device) != hipSuccess) return VCFC_E_HIP;
    const int fd = open(in_path, O_RDONLY);
    if (fd < 0) return VCFC_E_IO;
    auto sink = [&](const uint8_t *p, uint64_t k) {
        while (k) {
            const ssize_t w = write(out_fd, p, std::min<uint64_t>(k, 1ull << 30));
            if (w <= 0) return false;
            p += w;
            k -= (uint64_t)w;
        }
        return true;
    };
    vcfc_dec::SparseQuery q;
    q.ref = reinterpret_cast<const uint8_t *>(ref); q.ref_len = ref_len; q.has_range = has_range;
    q.start = start; q.end = end;
    CtxDecodeBuffers B(c);
    const int st = vcfc_dec::sparse_query(fd, q, B, c->stream, sink, (c->trace & VCFC_TRACE_SPARSE_QUERY) != 0);
    close(fd);
    return st;
}

int vcfc_query_match_device(const uint8_t *d_in, const uint64_t *d_rec_start, uint64_t n, const uint8_t *d_ref,
                            uint64_t ref_len, int has_range, uint64_t start, uint64_t end, uint8_t *d_flag,
                            uint64_t *d_err, void *stream) {
    if ((n && (!d_in || !d_rec_start || !d_flag)) || (!d_ref && ref_len) || ref_len > 0xFFFFFFFFull || !d_err)
        return VCFC_E_ARG;
    VcfcQuery q;
    q.ref = d_ref; q.ref_len = (uint32_t)ref_len; q.has_range = has_range ? 1u : 0u; q.start = start; q.end = end;
    return vcfc_query_match(d_in, d_rec_start, n, q, d_flag, d_err, static_cast<hipStream_t>(stream)) == hipSuccess
               ? VCFC_OK : VCFC_E_HIP;
}

int vcfc_record_hash_device(const uint8_t *d_recs, const uint64_t *d_rec_off, uint64_t n, uint64_t *d_hash,
                            void *stream) {
    if (n && (!d_recs || !d_rec_off || !d_hash)) return VCFC_E_ARG;
    return vcfc_record_hash(d_recs, d_rec_off, n, d_hash, static_cast<hipStream_t>(stream)) == hipSuccess
               ? VCFC_OK : VCFC_E_HIP;
}

uint64_t vcfc_decode_workspace_size(uint64_t n_records) { return vcfc_decode_workspace_layout(n_records).total; }

int vcfc_decode_selected_device(const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_rec_start,
                                const uint8_t *d_select, uint64_t n, uint64_t samples, uint8_t *d_out, uint64_t out_cap,
                                uint64_t *d_line_off, void *d_ws, uint64_t ws_bytes, uint64_t *d_err, int exact,
                                void *stream) {
    if ((n && (!d_in || !d_rec_start || !d_out || !d_ws)) || !d_line_off || !d_err) return VCFC_E_ARG;
    const VcfcDecodeLayout L = vcfc_decode_workspace_layout(n);
    if (ws_bytes < L.total) return VCFC_E_NOSPACE;
    uint8_t *ws = static_cast<uint8_t *>(d_ws);
    hipStream_t s = static_cast<hipStream_t>(stream);
    VcfcDecodeArgs a;
    a.in = d_in; a.n_bytes = in_bytes; a.rec_start = d_rec_start; a.select = d_select; a.n = n; a.S = samples;
    a.out = d_out; a.out_cap = out_cap; a.line_off = d_line_off;
    a.st = reinterpret_cast<uint32_t *>(ws + L.st);
    a.line_size = reinterpret_cast<uint32_t *>(ws + L.line_size);
    a.end = reinterpret_cast<uint64_t *>(ws + L.end);
    a.seq_list = reinterpret_cast<uint32_t *>(ws + L.seq_list);
    a.seq_count = reinterpret_cast<uint32_t *>(ws + L.seq_count);
    a.err = d_err;
    a.partials = reinterpret_cast<uint64_t *>(ws + L.partials);
    if (vcfc_decode_plan(a, exact != 0, s) != hipSuccess) return VCFC_E_HIP;
    return vcfc_decode_write(a, 0, n, s) == hipSuccess ? VCFC_OK : VCFC_E_HIP;
}

int vcfc_decode_records_device(const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_rec_start, uint64_t n,
                               uint64_t samples, uint8_t *d_out, uint64_t out_cap, uint64_t *d_line_off, void *d_ws,
                               uint64_t ws_bytes, uint64_t *d_err, int exact, void *stream) {
    return vcfc_decode_selected_device(d_in, in_bytes, d_rec_start, nullptr, n, samples, d_out, out_cap, d_line_off,
                                       d_ws, ws_bytes, d_err, exact, stream);
}

}  // extern "C"
