// TEST INFRASTRUCTURE ONLY: C entry point that runs the product encode
// pipeline (vcfc_encode_device from csrc/vcfc_encode.hip) on the fiber
// emulator, with host memory standing in for HBM.
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#include "vcfc_device.h"
#include "vcfc_decode_driver.h"
#include "emu.h"
#include <atomic>

// bytes the hop line index's walkers loaded (VCFC_DIAG_HOP_READ, diag_retries.h)
static std::atomic<unsigned long long> g_hop_read{0};
void emu_diag_hop_read(unsigned long long bytes) { g_hop_read += bytes; }
extern "C" unsigned long long emu_hop_read(int reset) {
    const unsigned long long v = g_hop_read.load();
    if (reset) g_hop_read = 0;
    return v;
}

static uint32_t g_last_deferred = 0;
// deferred records: EMU_DEFER=0 / 1 forces them off / on, else the product default
static uint32_t emu_defer() {
    const char *e = getenv("EMU_DEFER");
    return e ? (atoi(e) != 0 ? 1u : 0u) : (uint32_t)VCFC_DEFER_DEFAULT;
}
static uint32_t g_last_mispredict = 0;
// rows the last emu_encode_rows call deferred (VCFCD_DEFER: written by
// k_encode_defer; predicted rows taken by the general path after all not counted)
extern "C" uint32_t emu_last_deferred() { return g_last_deferred; }
// whether its first deferred pass found a predicted size wrong (the layout ran again)
extern "C" uint32_t emu_last_mispredict() { return g_last_mispredict; }

extern "C" int emu_encode_rows(const uint8_t *buf, const uint64_t *line_off, const uint32_t *line_len,
                               uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *rec_off,
                               uint64_t *err_word, uint64_t *switches, uint32_t *retries) {
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; i++) total += line_len[i];
    VcfcWorkspaceLayout L = vcfc_encode_workspace_layout(n, total);
    uint8_t *ws = (uint8_t *)aligned_alloc(256, (L.total + 255) & ~255ull);
    memset(ws, 0xCD, L.total);  // poison: stale workspace must not leak into results
    VcfcEncodeArgs a;
    a.buf = buf; a.line_off = line_off; a.line_len = line_len; a.n = n;
    a.out = out; a.out_cap = out_cap; a.rec_off = rec_off;
    vcfc_encode_args_workspace(a, ws, L);
    a.line_bytes_hint = getenv("EMU_WIDE_COMPACT") ? (~0ull >> 1) : total;   // (tests force the 64-lane compaction)
    a.err = (uint64_t *)(ws + L.err);
    a.defer_records = emu_defer();   // (tests: deferred records; the product default unless EMU_DEFER is set)
    a.nl_check = getenv("EMU_NL_CHECK") ? 1u : 0u;   // (tests: rows from a guessed line index)
    emu::g.switches = 0;
    int st = (int)vcfc_encode_device(a, nullptr);
    *err_word = *a.err;
    if (retries) *retries = *a.retry_count;   // rows that took the general path
    g_last_deferred = *a.defer_count - *a.defer_fallback;
    g_last_mispredict = *a.mispredict;
    if (switches) *switches = emu::g.switches;
    free(ws);
    return st;
}

hipError_t vcfc_sparse_plan_launch(const uint8_t *recs, const uint64_t *rec_off, uint64_t n, uint64_t data_start,
                                   uint64_t *file_off, uint8_t *prefix, uint64_t *status, hipStream_t s);

extern "C" int emu_sparse_plan(const uint8_t *recs, const uint64_t *rec_off, uint64_t n, uint64_t data_start,
                               uint64_t *file_off, uint8_t *prefix, uint64_t *status) {
    return (int)vcfc_sparse_plan_launch(recs, rec_off, n, data_start, file_off, prefix, status, nullptr);
}

// The product decode driver (csrc/vcfc_decode_driver.h) over host memory:
// header parse + decode_section with small output batches (exercises the
// batching).  Returns the driver status; *out_len = bytes produced.
namespace {
struct HostBuffers : vcfc_dec::Buffers {
    std::vector<uint8_t> b[N_SLOTS];
    void *get(int slot, uint64_t bytes) override {
        if (b[slot].size() < bytes) b[slot].assign(bytes, 0xCD);   // poison
        return b[slot].data();
    }
};
}  // namespace

extern "C" int emu_decompress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len,
                              uint64_t out_batch) {
    uint64_t data_off = 0, S = 0;
    *out_len = 0;
    int st = vcfc_dec::parse_header(in, n, &data_off, &S);
    if (st) return st;
    uint64_t o = 0;
    auto sink = [&](const uint8_t *p, uint64_t k) {
        if (o + k > cap) return false;
        memcpy(out + o, p, k);
        o += k;
        return true;
    };
    sink(in, data_off);
    HostBuffers B;
    st = vcfc_dec::decode_section(in + data_off, n - data_off, S, B, nullptr, sink, out_batch);
    *out_len = o;
    return st;
}

// Range query through the product driver (vcfc_dec::query_section).
extern "C" int emu_query(const uint8_t *in, uint64_t n, const uint8_t *ref, uint64_t ref_len, int has_range,
                         uint64_t qstart, uint64_t qend, uint8_t *out, uint64_t cap, uint64_t *out_len,
                         uint64_t out_batch) {
    uint64_t data_off = 0, S = 0;
    *out_len = 0;
    int st = vcfc_dec::parse_header(in, n, &data_off, &S);
    if (st) return st;
    uint64_t o = 0;
    auto sink = [&](const uint8_t *p, uint64_t k) {
        if (o + k > cap) return false;
        memcpy(out + o, p, k);
        o += k;
        return true;
    };
    HostBuffers B;
    st = vcfc_dec::query_section(in + data_off, n - data_off, S, ref, ref_len, has_range, qstart, qend, B, nullptr,
                                 sink, out_batch);
    *out_len = o;
    return st;
}

// Sparse-file query through the product driver (vcfc_dec::sparse_query) on a
// real file; lines to out_fd.
#include <fcntl.h>
extern "C" int emu_sparse_query(const char *path, const uint8_t *ref, uint64_t ref_len, int has_range,
                                uint64_t qstart, uint64_t qend, int out_fd) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return vcfc_dec::ST_E_IO;
    auto sink = [&](const uint8_t *p, uint64_t k) { return write(out_fd, p, k) == (ssize_t)k; };
    vcfc_dec::SparseQuery q;
    q.ref = ref; q.ref_len = ref_len; q.has_range = has_range; q.start = qstart; q.end = qend;
    HostBuffers B;
    const int st = vcfc_dec::sparse_query(fd, q, B, nullptr, sink);
    close(fd);
    return st;
}

// Pipelined compress() through the product driver (vcfc_ing::compress_stream)
// with a small chunk size, so carries across chunks and the '#' line
// interleave are exercised on small inputs.
#include "vcfc_ingest_driver.h"
namespace {
struct HostIngestMemory : vcfc_ing::Memory {
    std::vector<uint8_t> d[N_DEV], h[N_HOST];
    void *dev(int slot, uint64_t bytes) override {
        if (d[slot].size() < bytes + 16) d[slot].assign(bytes + 16, 0xCD);   // poison
        return d[slot].data();
    }
    void *host(int slot, uint64_t bytes) override {
        if (h[slot].size() < bytes + 16) h[slot].assign(bytes + 16, 0xCD);
        return h[slot].data();
    }
};
struct BufSource : vcfc_ing::Source {
    const uint8_t *p;
    uint64_t n;
    uint64_t size() const override { return n; }
    bool read(uint8_t *dst, uint64_t off, uint64_t k) override {
        memcpy(dst, p + off, k);
        return true;
    }
};
}  // namespace

extern "C" int emu_compress(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len,
                            int64_t *err_line, uint64_t chunk, int read_threads, uint64_t max_chunk) {
    uint64_t o = 0;
    auto sink = [&](const uint8_t *p, uint64_t k) {
        if (o + k > cap) return false;
        memcpy(out + o, p, k);
        o += k;
        return true;
    };
    BufSource src;
    src.p = in;
    src.n = n;
    HostIngestMemory M;
    vcfc_ing::Config cfg;
    cfg.chunk = chunk;
    cfg.read_threads = read_threads;
    if (max_chunk) cfg.max_chunk = max_chunk;
    int st = vcfc_ing::compress_stream(src, sink, M, nullptr, cfg, err_line);
    *out_len = o;
    return st;
}

// compress() of "device-resident" bytes (host memory on the emulator)
// through vcfc_ing::compress_device, with small chunks.
extern "C" int emu_compress_device(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len,
                                   int64_t *err_line, uint64_t chunk, uint64_t max_chunk, int hop,
                                   uint64_t *hop_redo) {
    HostIngestMemory M;
    vcfc_ing::Config cfg;
    cfg.chunk = chunk;
    if (max_chunk) cfg.max_chunk = max_chunk;
    cfg.hop_index = hop != 0;            // hop: 0 scan, 1 hop (learning when the first lines need it),
    cfg.hop_learn = hop == 2 ? 1 : hop == 3 ? 0 : -1;   // 2 hop learning, 3 hop without learning
    cfg.hop_redo = hop_redo;
    cfg.defer_records = emu_defer() != 0;
    return vcfc_ing::compress_device(in, n, out, cap, out_len, M, nullptr, cfg, err_line);
}

// Per-record digests (csrc/vcfc_check.hip) on the emulator.
extern "C" int emu_record_hash(const uint8_t *recs, const uint64_t *rec_off, uint64_t n, uint64_t *out) {
    return (int)vcfc_record_hash(recs, rec_off, n, out, nullptr);
}

// Synthetic rows (csrc/vcfc_synth.hip) on the emulator.
hipError_t vcfc_synth_device(uint8_t *buf, const uint64_t *line_off, uint64_t n, const uint8_t *prefix,
                             const uint64_t *prefix_off, const float *row_af, uint32_t S, int law,
                             uint64_t seed, uint64_t row_base, hipStream_t s);
extern "C" int emu_synth(uint8_t *buf, const uint64_t *line_off, uint64_t n, const uint8_t *prefix,
                         const uint64_t *prefix_off, const float *row_af, uint32_t S, int law, uint64_t seed,
                         uint64_t row_base) {
    return (int)vcfc_synth_device(buf, line_off, n, prefix, prefix_off, row_af, S, law, seed, row_base, nullptr);
}

// vcfc_ing::Held (the held output of a sharded compress rank): append `n`
// bytes in pieces of `piece`, with the first mem_bound bytes in memory and
// the rest spilled to a file in `dir`; then place them at out_off of out_fd.
extern "C" int emu_held(const uint8_t *data, uint64_t n, uint64_t piece, uint64_t mem_bound, const char *dir,
                        int out_fd, uint64_t out_off, uint64_t *mem_bytes, uint64_t *spill_bytes) {
    vcfc_ing::Held h;
    h.mem_bound = mem_bound;
    h.spill_dir = dir;
    for (uint64_t o = 0; o < n; o += piece)
        if (!h.append(data + o, std::min<uint64_t>(piece, n - o))) return 7;
    *mem_bytes = h.mem;
    *spill_bytes = h.spilled;
    return h.place(out_fd, out_off) ? 0 : 7;
}

// The line index (csrc/vcfc_ingest.hip) of in[0, n) (last byte '\n'): the
// data lines' offsets and lengths and the counts; S_hint != 0: the hop index
// (learn: its TRY / LEARN walkers, else the GUESS ones; len_hint: their
// first guess, compress_device's first data line length).
extern "C" int emu_line_index(const uint8_t *in, uint64_t n, uint32_t S_hint, uint64_t *off, uint32_t *len,
                              uint64_t cap, uint64_t *counts, uint64_t hop_walkers, int learn, uint32_t len_hint) {
    const VcfcLineIndexLayout L1 = vcfc_line_index_layout(n, 0);
    std::vector<uint8_t> ws1(L1.total1 + 64);
    std::vector<uint64_t> cnt(4, 0);
    VcfcLineIndex x;
    memset(&x, 0, sizeof x);
    x.counts = cnt.data();
    if (vcfc_line_index(in, n, ws1.data(), L1, x, nullptr, S_hint, hop_walkers, learn != 0, len_hint) != hipSuccess) return 1;
    const uint64_t lines = cnt[0];
    const VcfcLineIndexLayout L = vcfc_line_index_layout(n, lines);
    std::vector<uint8_t> ws2(L.total2 + 64);
    std::vector<uint64_t> lo(lines + 1), po(lines + 1), pb(lines + 1);
    std::vector<uint32_t> ll(lines + 1), ln(lines + 1), pl(lines + 1), pn(lines + 1);
    x.line_off = lo.data(); x.line_len = ll.data(); x.line_no = ln.data();
    x.pass_off = po.data(); x.pass_len = pl.data(); x.pass_no = pn.data(); x.pass_before = pb.data();
    if (vcfc_line_index_place(in, n, lines, ws1.data(), ws2.data(), L, x, nullptr) != hipSuccess) return 1;
    memcpy(counts, cnt.data(), 32);
    const uint64_t k = std::min<uint64_t>(cnt[1], cap);
    memcpy(off, lo.data(), 8 * k);
    memcpy(len, ll.data(), 4 * k);
    return 0;
}

// compress_device's choice of the hop index's learning (host code)
extern "C" int emu_data_lines_irregular(const uint8_t *p, uint64_t len, uint32_t S) {
    return vcfc_ing::data_lines_irregular(p, len, S) ? 1 : 0;
}
