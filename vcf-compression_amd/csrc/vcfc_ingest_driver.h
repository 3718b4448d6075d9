// vcfc_ingest_driver.h -- pipelined compress(), shared by
// the C ABI (vcfc_api.cpp) and the CPU emulator harness
// (tests/simt_emu/emu_api.cpp), so the same control flow is tested on both.
//
// Reference: compress() (src/compress.cpp:205-257) reads the VCF with
// getline, copies '#' lines through with '\n', skips empty lines, encodes
// data lines with compress_data_line and stops at the first line that
// throws.  Here three stages run concurrently on fixed-size chunks of whole
// lines:
//
//   reader  (host threads)  the input in chunks of up to `chunk` bytes into
//                           pinned host slots; the partial line at a chunk's
//                           end is carried to the next chunk;
//   uploader (host thread)  H2D of each chunk into one of two device slots on
//                           its own stream, so the copy of chunk k+1 overlaps
//                           the GPU work on chunk k;
//   GPU     (calling thread) line index (vcfc_ingest.hip) -> encode
//                           (vcfc_encode.hip) -> D2H of the records, the
//                           '#' lines checked on the host (>= 8 terms);
//   writer  (host thread)   records with the '#' lines interleaved at their
//                           places, in input order.
//
// The output equals the reference's up to the first failing line; that
// line's status and 1-based number are returned.
#pragma once
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fcntl.h>
#include <unistd.h>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "vcfc_device.h"
#include "vcfc_queue.h"

namespace vcfc_ing {

// = include/vcfc.h codes
constexpr int ST_OK = 0, ST_E_LT8COLS = 1, ST_E_8COLS = 2, ST_E_HEADER = 3, ST_E_NOSPACE = 4, ST_E_ARG = 5,
              ST_E_HIP = 6, ST_E_IO = 7;

// Input bytes [off, off + n) into dst; must be safe to call from several
// threads at once.  false = I/O error.
struct Source {
    virtual ~Source() {}
    virtual uint64_t size() const = 0;
    virtual bool read(uint8_t *dst, uint64_t off, uint64_t n) = 0;
};
// In-order output; false = I/O error (or no space).
using Sink = std::function<bool(const uint8_t *, uint64_t)>;

// Output held for a later placement (a rank of a sharded compress whose file
// offset is known only after the all-gather of the ranks' byte counts): the
// first mem_bound bytes in host memory (64 MiB blocks), the rest appended to
// a spill file (unlinked at once; only its fd is kept).  place() writes the
// held bytes at the given file offset: one pwrite per memory block, the spill
// part copied in-kernel (copy_file_range) or by pread/pwrite -- so the bytes
// that fit in memory are written once, to their final place.
struct Held {
    static constexpr uint64_t BLOCK = 64ull << 20;
    std::vector<std::unique_ptr<uint8_t[]>> blocks;
    uint64_t mem_bound = 0, mem = 0, spilled = 0;
    std::string spill_dir;
    int spill_fd = -1;
    ~Held() {
        if (spill_fd >= 0) close(spill_fd);
    }
    uint64_t bytes() const { return mem + spilled; }
    bool append(const uint8_t *p, uint64_t k) {
        while (k && mem < mem_bound) {
            if (mem / BLOCK >= blocks.size()) {
                blocks.emplace_back(new (std::nothrow) uint8_t[BLOCK]);
                if (!blocks.back()) return false;
            }
            const uint64_t at = mem % BLOCK;
            const uint64_t take = std::min<uint64_t>({k, BLOCK - at, mem_bound - mem});
            memcpy(blocks[mem / BLOCK].get() + at, p, take);
            p += take; k -= take; mem += take;
        }
        if (!k) return true;
        if (spill_fd < 0) {
            std::string path = (spill_dir.empty() ? std::string("/tmp") : spill_dir) + "/.vcfc-held-XXXXXX";
            std::vector<char> t(path.begin(), path.end());
            t.push_back('\0');
            spill_fd = mkstemp(t.data());
            if (spill_fd < 0) return false;
            unlink(t.data());
        }
        while (k) {
            const ssize_t w = pwrite(spill_fd, p, std::min<uint64_t>(k, 1ull << 30), (off_t)spilled);
            if (w <= 0) return false;
            p += w; k -= (uint64_t)w; spilled += (uint64_t)w;
        }
        return true;
    }
    bool place(int fd, uint64_t off) const {
        auto put = [&](const uint8_t *b, uint64_t k, uint64_t at) {
            while (k) {
                const ssize_t w = pwrite(fd, b, std::min<uint64_t>(k, 1ull << 30), (off_t)at);
                if (w <= 0) return false;
                b += w; k -= (uint64_t)w; at += (uint64_t)w;
            }
            return true;
        };
        for (uint64_t q = 0; q * BLOCK < mem; q++)
            if (!put(blocks[q].get(), std::min(BLOCK, mem - q * BLOCK), off + q * BLOCK)) return false;
        uint64_t done = 0;
        while (done < spilled) {   // in-kernel copy where the filesystems allow it
            loff_t si = (loff_t)done, di = (loff_t)(off + mem + done);
            const ssize_t c = copy_file_range(spill_fd, &si, fd, &di, spilled - done, 0);
            if (c <= 0) break;
            done += (uint64_t)c;
        }
        std::vector<uint8_t> tmp;
        while (done < spilled) {
            tmp.resize(std::min<uint64_t>(spilled - done, 64ull << 20));
            const ssize_t r = pread(spill_fd, tmp.data(), tmp.size(), (off_t)done);
            if (r <= 0 || !put(tmp.data(), (uint64_t)r, off + mem + done)) return false;
            done += (uint64_t)r;
        }
        return true;
    }
};

// Device and pinned host buffers, owned by the caller; contents not kept
// between calls.
struct Memory {
    virtual ~Memory() {}
    enum { D_IN0 = 0, D_IN1, D_IX1, D_IX2, D_LINES, D_ENC_WS, D_OUT, D_REC, D_SMALL, N_DEV };
    enum { H_IN0 = 0, H_IN1, H_IN2, H_OUT0, H_OUT1, H_SMALL, N_HOST };
    virtual void *dev(int slot, uint64_t bytes) = 0;    // nullptr on failure
    virtual void *host(int slot, uint64_t bytes) = 0;   // pinned; nullptr on failure
};

struct Config {
    uint64_t chunk = 256ull << 20;   // input bytes per chunk; a chunk grows to hold a longer line
    uint64_t max_chunk = 3ull << 30; // growth limit (line offsets in a chunk are 32-bit; a record's
                                     // LEN header holds < 2^30 anyway, reference src/utils.hpp:160)
    int read_threads = 8;
    bool hop_index = true;           // compress_device: the hop line index (S from "#CHROM")
    int hop_learn = -1;              // ... learning other region lengths: -1 = when the first data lines need it
    uint64_t hop_walkers = 0;        // ... walkers (0: the kernel's count; tests)
    bool trace = false;              // stage totals / decisions to stderr (vcfc_ctx_set_trace)
    bool defer_records = false;      // VcfcEncodeArgs::defer_records (vcfc_ctx_set_deferred_records)
    uint64_t *hop_redo = nullptr;    // compress_device: chunks indexed again after a wrong hop guess
};

// compress()'s header-line check (src/compress.cpp:230-235): split_string
// drops empty terms (src/utils.cpp:82-116), and fewer than 8 throw.
inline bool header_ok(const uint8_t *p, uint64_t len) {
    uint64_t terms = 0, q = 0;
    while (q < len) {
        while (q < len && p[q] == '\t') q++;
        if (q >= len) break;
        terms++;
        while (q < len && p[q] != '\t') q++;
    }
    return terms >= 8;
}

// Samples of the "#CHROM" line held whole in p[0, len) (TABs - 8), 0 if none:
// only a guess for the hop line index, never trusted for the output.
// *more: the window ended inside the header (a longer one may hold it).
inline uint32_t header_samples(const uint8_t *p, uint64_t len, bool *more = nullptr) {
    static const char key[] = "#CHROM\t";
    if (more) *more = false;
    for (uint64_t q = 0; q < len;) {
        const uint8_t *e = static_cast<const uint8_t *>(memchr(p + q, '\n', len - q));
        if (!e) {
            if (more) *more = p[q] == '#';
            return 0;
        }
        const uint64_t end = (uint64_t)(e - p);
        if (end - q >= 7 && memcmp(p + q, key, 7) == 0) {
            uint64_t tabs = 0;
            for (uint64_t k = q; k < end; k++) tabs += p[k] == '\t';
            return tabs >= 9 && tabs - 8 < (1u << 24) ? (uint32_t)(tabs - 8) : 0u;
        }
        if (end > q && p[q] != '#') return 0;   // the header ended (empty lines are skipped)
        q = end + 1;
    }
    if (more) *more = len > 0;   // the window ended at a line end inside the header
    return 0;
}

// Whether the complete data lines in p[0, len) after the "#CHROM" line hold
// anything but S 3-byte tokens (genotype region != 4 S - 1 bytes): then the
// hop line index learns other region lengths (vcfc_line_index hop_learn).
// Only a guess, never trusted for the output.
inline bool data_lines_irregular(const uint8_t *p, uint64_t len, uint32_t S) {
    bool in_data = false;
    for (uint64_t q = 0; q < len;) {
        const uint8_t *nl = static_cast<const uint8_t *>(memchr(p + q, '\n', len - q));
        if (!nl) break;
        const uint64_t end = (uint64_t)(nl - p);
        if (!in_data) {
            in_data = end - q >= 7 && memcmp(p + q, "#CHROM\t", 7) == 0;
        } else if (end > q && p[q] != '#') {
            uint64_t k = q;
            for (uint32_t t = 0; t < 9 && k < end; k++) t += p[k] == '\t';
            if (end - k != 4ull * S - 1) return true;
        }
        q = end + 1;
    }
    return false;
}

// The length (with its '\n') of the first data line after "#CHROM" that lies
// whole in p[0, len), or 0: the hop index's first guess (vcfc_line_index
// len_hint) for every walker's first line.
inline uint32_t first_data_line_len(const uint8_t *p, uint64_t len) {
    bool in_data = false;
    for (uint64_t q = 0; q < len;) {
        const uint8_t *nl = static_cast<const uint8_t *>(memchr(p + q, '\n', len - q));
        if (!nl) break;
        const uint64_t end = (uint64_t)(nl - p);
        if (!in_data) {
            in_data = end - q >= 7 && memcmp(p + q, "#CHROM\t", 7) == 0;
        } else if (end > q && p[q] != '#') {
            return end + 1 - q < (1ull << 30) ? (uint32_t)(end + 1 - q) : 0u;
        }
        q = end + 1;
    }
    return 0;
}

// The TRY / LEARN walkers' first candidates (VcfcHopCands): the data lines
// of p[0, len) after "#CHROM" whose genotype region (after the 9th TAB, up
// to the '\n') is not 4 S - 1 bytes and at least 255 -- up to three distinct
// region lengths, each with the TAB masks of the 256 bytes ending at its
// '\n', exactly what a walker's LEARN takes from such a line.
inline void learn_candidates(const uint8_t *p, uint64_t len, uint32_t S, VcfcHopCands *c) {
    memset(c, 0, sizeof *c);
    uint32_t k = 0;
    bool in_data = false;
    for (uint64_t q = 0; q < len && k < 3;) {
        const uint8_t *nl = static_cast<const uint8_t *>(memchr(p + q, '\n', len - q));
        if (!nl) break;
        const uint64_t end = (uint64_t)(nl - p);
        if (!in_data) {
            in_data = end - q >= 7 && memcmp(p + q, "#CHROM\t", 7) == 0;
        } else if (end > q && p[q] != '#') {
            uint64_t t = q;
            uint32_t tabs = 0;
            for (; t < end && tabs < 9; t++) tabs += p[t] == '\t';
            const uint64_t G = end - t;   // t: the first sample byte (when 9 TABs were found)
            if (tabs == 9 && G != 4ull * S - 1 && G >= 255 && G < (1ull << 31) && G != c->g[0] && G != c->g[1]) {
                const uint64_t g0 = end + 1 - 256;
                for (uint32_t wl = 0; wl < 16; wl++) {
                    uint32_t m = 0;
                    for (uint32_t j = 0; j < 16; j++) m |= (p[g0 + 16 * wl + j] == '\t' ? 1u : 0u) << j;
                    c->sig[k][wl] = (uint16_t)m;
                }
                c->g[k++] = (uint32_t)G;
            }
        }
        q = end + 1;
    }
}

namespace detail {

inline double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

using vcfc_q::Queue;   // bounded hand-off between the stages

struct InChunk {
    int slot = -1;
    int dslot = -1;       // device copy (set by the uploader)
    uint8_t *host = nullptr;       // pinned copy (slot `slot`)
    const uint8_t *dev = nullptr;  // device copy (slot `dslot`)
    uint64_t bytes = 0;   // whole lines, the last one ending with '\n'
    bool ok = true;       // false: read or allocation error, or a line longer than cfg.max_chunk
    bool long_line = false;
    bool alloc_failed = false;
};

struct PassLine {
    uint64_t before;   // data lines of the chunk before it
    uint32_t no;       // line number in the chunk
    std::vector<uint8_t> text;
};

struct OutChunk {
    int slot = -1;
    const uint8_t *data = nullptr;        // pinned records (slot `slot`)
    uint64_t rec_bytes = 0;               // records of the good rows
    std::vector<uint64_t> rec_off;        // only when pass lines are interleaved
    std::vector<PassLine> pass;           // the ones to write
    bool last = false;
};

}  // namespace detail

// Compress `src` into `sink`.  *err_line = 1-based line of the failing line
// (-1 if none); *lines_out = lines consumed ('\n'-terminated, an unterminated
// last line counts as one) when the whole input was compressed.  Chunks hold cfg.chunk bytes of whole lines; a line longer
// than that grows its chunk (doubling) until the line fits, so no input is
// read twice.  ST_E_ARG: a line longer than cfg.max_chunk (the lines before
// it have been written).  Every buffer is sized per chunk: the pinned output
// slots by the chunk's actual record bytes.
inline int compress_stream(Source &src, const Sink &sink, Memory &M, hipStream_t s, const Config &cfg,
                           int64_t *err_line, uint64_t *lines_out = nullptr) {
    using namespace detail;
    if (err_line) *err_line = -1;
    if (lines_out) *lines_out = 0;
    const uint64_t N = src.size();
    const uint64_t C = cfg.chunk;
    if (N == 0) return ST_OK;
    if (C < 16 || C > cfg.max_chunk) return ST_E_ARG;
    uint8_t *hin[3];
    uint64_t hin_cap[3];
    for (int k = 0; k < 3; k++) {
        hin_cap[k] = C + 64;   // + the '\n' after an unterminated last line
        if (!(hin[k] = static_cast<uint8_t *>(M.host(Memory::H_IN0 + k, hin_cap[k])))) return ST_E_HIP;
    }
    uint8_t *hout[2] = {nullptr, nullptr};
    uint64_t hout_cap[2] = {0, 0};
    uint64_t *hsmall = static_cast<uint64_t *>(M.host(Memory::H_SMALL, 64));
    uint8_t *d_inb[2] = {nullptr, nullptr};
    uint64_t d_inb_cap[2] = {0, 0};
    uint64_t *d_small = static_cast<uint64_t *>(M.dev(Memory::D_SMALL, 64));
    if (!hsmall || !d_small) return ST_E_HIP;
    hipStream_t s_copy = nullptr;
    hipEvent_t ev_up[2] = {nullptr, nullptr};
    if (hipStreamCreateWithFlags(&s_copy, hipStreamNonBlocking) != hipSuccess) return ST_E_HIP;
    if (hipEventCreateWithFlags(&ev_up[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ev_up[1], hipEventDisableTiming) != hipSuccess) {
        for (hipEvent_t e : ev_up)
            if (e) (void)hipEventDestroy(e);
        (void)hipStreamDestroy(s_copy);
        return ST_E_HIP;
    }

    // ---- reader ------------------------------------------------------------
    Queue<InChunk> filled;
    Queue<int> free_in;
    for (int k = 0; k < 3; k++) free_in.put(k);
    std::vector<uint8_t> carry;
    const bool trace = cfg.trace;
    double t_read = 0, t_gpu = 0, t_write = 0, t_wait_in = 0, t_wait_out = 0;
    const double t_begin = now_s();
    std::thread reader([&] {
        uint64_t pos = 0;
        // read [pos, pos + want) into b + at with up to cfg.read_threads threads
        auto read_into = [&](uint8_t *b, uint64_t at, uint64_t want) {
            const int T = want >= (1u << 20) ? std::max(1, cfg.read_threads) : 1;
            std::vector<std::thread> ts;
            std::vector<char> ok(T, 1);
            const uint64_t per = (want + T - 1) / T;
            for (int t = 0; t < T; t++) {
                const uint64_t a = t * per, e = std::min(want, a + per);
                if (a >= e) continue;
                ts.emplace_back([&, t, a, e] { ok[t] = src.read(b + at + a, pos + a, e - a) ? 1 : 0; });
            }
            const double r0 = now_s();
            for (auto &t : ts) t.join();
            t_read += now_s() - r0;
            bool all = true;
            for (char o : ok) all = all && o;
            pos += want;
            return all;
        };
        while (pos < N) {
            int slot;
            if (!free_in.get(slot)) break;
            InChunk ch;
            ch.slot = slot;
            uint8_t *b = hin[slot];
            const uint64_t c0 = carry.size();
            uint64_t lim = std::max<uint64_t>(C, c0);   // chunk bytes this time
            if (lim + 64 > hin_cap[slot]) {
                if (!(b = static_cast<uint8_t *>(M.host(Memory::H_IN0 + slot, lim + 64)))) {
                    ch.ok = false; ch.alloc_failed = true;
                    filled.put(ch);
                    break;
                }
                hin[slot] = b;
                hin_cap[slot] = lim + 64;
            }
            if (c0) memcpy(b, carry.data(), c0);
            uint64_t total = c0;
            uint64_t scanned = c0;   // bytes [0, scanned) hold no '\n' (carry holds none)
            const uint8_t *nl = nullptr;
            for (;;) {
                const uint64_t want = std::min<uint64_t>(lim - total, N - pos);
                ch.ok = read_into(b, total, want) && ch.ok;
                total += want;
                if (pos >= N || !ch.ok) break;
                nl = static_cast<const uint8_t *>(memrchr(b + scanned, '\n', total - scanned));
                if (nl) break;
                scanned = total;
                // a line longer than the chunk: double the chunk, keep its bytes
                if (lim >= cfg.max_chunk) { ch.ok = false; ch.long_line = true; break; }
                const uint64_t grown = std::min<uint64_t>(2 * lim, cfg.max_chunk);
                std::vector<uint8_t> keep(b, b + total);
                if (!(b = static_cast<uint8_t *>(M.host(Memory::H_IN0 + slot, grown + 64)))) {
                    ch.ok = false; ch.alloc_failed = true;
                    break;
                }
                memcpy(b, keep.data(), total);
                hin[slot] = b;
                hin_cap[slot] = grown + 64;
                lim = grown;
            }
            ch.host = b;
            carry.clear();
            if (ch.ok && pos >= N) {
                if (total && b[total - 1] != '\n') b[total++] = '\n';   // getline returns an unterminated last line
                ch.bytes = total;
            } else if (ch.ok) {
                ch.bytes = (uint64_t)(nl - b) + 1;
                carry.assign(b + ch.bytes, b + total);
            }
            filled.put(ch);
            if (!ch.ok) break;
        }
        filled.close();
    });

    // ---- uploader ------------------------------------------------------------
    Queue<InChunk> uploaded;
    Queue<int> free_dev;
    free_dev.put(0);
    free_dev.put(1);
    std::thread uploader([&] {
        InChunk ch;
        while (filled.get(ch)) {
            if (ch.ok) {
                int ds;
                if (!free_dev.get(ds)) break;
                ch.dslot = ds;
                if (ch.bytes + 64 > d_inb_cap[ds]) {   // first use, or a grown chunk
                    d_inb[ds] = static_cast<uint8_t *>(M.dev(Memory::D_IN0 + ds, ch.bytes + 64));
                    d_inb_cap[ds] = d_inb[ds] ? ch.bytes + 64 : 0;
                }
                ch.dev = d_inb[ds];
                if (!ch.dev || hipMemcpyAsync(d_inb[ds], ch.host, ch.bytes, hipMemcpyHostToDevice, s_copy) != hipSuccess ||
                    hipEventRecord(ev_up[ds], s_copy) != hipSuccess)
                    ch.ok = false;
            }
            uploaded.put(ch);
            if (!ch.ok) break;
        }
        uploaded.close();
    });

    // ---- writer ------------------------------------------------------------
    Queue<OutChunk> to_write;
    Queue<int> free_out;
    free_out.put(0);
    free_out.put(1);
    bool write_failed = false;
    std::thread writer([&] {
        OutChunk oc;
        while (to_write.get(oc)) {
            const uint8_t *r = oc.data;
            const double w0 = now_s();
            if (!write_failed) {
                if (oc.pass.empty()) {
                    if (oc.rec_bytes && !sink(r, oc.rec_bytes)) write_failed = true;
                } else {
                    uint64_t at = 0;   // records written so far
                    for (const PassLine &p : oc.pass) {
                        const uint64_t upto = oc.rec_off[p.before];
                        if (upto > at && !sink(r + at, upto - at)) { write_failed = true; break; }
                        at = std::max(at, upto);
                        if (!sink(p.text.data(), p.text.size())) { write_failed = true; break; }
                    }
                    if (!write_failed && oc.rec_bytes > at && !sink(r + at, oc.rec_bytes - at)) write_failed = true;
                }
            }
            t_write += now_s() - w0;
            free_out.put(oc.slot);
        }
    });

    // ---- GPU stage (this thread) --------------------------------------------
    int status = ST_OK;
    uint64_t line_base = 0;   // lines of the chunks before
    auto finish = [&](int st) {
        status = st;
        free_in.close();
        free_dev.close();
        filled.close();
        to_write.close();
        reader.join();
        uploader.join();
        writer.join();
        (void)hipStreamSynchronize(s_copy);
        (void)hipEventDestroy(ev_up[0]);
        (void)hipEventDestroy(ev_up[1]);
        (void)hipStreamDestroy(s_copy);
        if (status == ST_OK && write_failed) status = ST_E_IO;
        if (trace)
            fprintf(stderr, "vcfc ingest: %.3f s total; read %.3f s, gpu stage %.3f s (waiting for input %.3f s, "
                            "for an output slot %.3f s), write %.3f s\n",
                    now_s() - t_begin, t_read, t_gpu, t_wait_in, t_wait_out, t_write);
        return status;
    };
    auto sync = [&]() { return hipStreamSynchronize(s) == hipSuccess; };
    InChunk ch;
    for (;;) {
        double g0 = now_s();
        if (!uploaded.get(ch)) break;
        t_wait_in += now_s() - g0;
        g0 = now_s();
        struct Acc {
            double &t, g;
            ~Acc() { t += now_s() - g; }
        } acc{t_gpu, g0};
        if (!ch.ok) return finish(ch.long_line ? ST_E_ARG : (ch.alloc_failed || ch.dslot >= 0) ? ST_E_HIP : ST_E_IO);
        const uint64_t n = ch.bytes;
        const uint8_t *h = ch.host;
        const uint8_t *d_in = ch.dev;
        const VcfcLineIndexLayout L1 = vcfc_line_index_layout(n, 0);
        uint8_t *d_ix1 = static_cast<uint8_t *>(M.dev(Memory::D_IX1, L1.total1));
        if (!d_ix1) return finish(ST_E_HIP);
        VcfcLineIndex x;
        x.counts = d_small;
        // phase 1: '\n' positions
        if (hipStreamWaitEvent(s, ev_up[ch.dslot], 0) != hipSuccess ||
            vcfc_line_index(d_in, n, d_ix1, L1, x, s) != hipSuccess ||
            hipMemcpyAsync(hsmall, d_small, 8, hipMemcpyDeviceToHost, s) != hipSuccess || !sync())
            return finish(ST_E_HIP);
        const uint64_t n_lines = hsmall[0];
        // phase 2: data and '#' lines
        const VcfcLineIndexLayout L = vcfc_line_index_layout(n, n_lines);
        const uint64_t max_data = n_lines;
        uint8_t *d_ix2 = static_cast<uint8_t *>(M.dev(Memory::D_IX2, L.total2));
        uint8_t *d_lines = static_cast<uint8_t *>(M.dev(Memory::D_LINES, 32 * (max_data + 1)));
        if (!d_ix2 || !d_lines) return finish(ST_E_HIP);
        uint8_t *q = d_lines;
        x.line_off = reinterpret_cast<uint64_t *>(q); q += 8 * (max_data + 1);
        x.pass_before = reinterpret_cast<uint64_t *>(q); q += 8 * (max_data + 1);
        x.line_len = reinterpret_cast<uint32_t *>(q); q += 4 * (max_data + 1);
        x.line_no = reinterpret_cast<uint32_t *>(q); q += 4 * (max_data + 1);
        std::vector<uint32_t> pass_len, pass_no;
        std::vector<uint64_t> pass_off, pass_before;
        // the pass arrays (off, len, no) share one buffer with the record offsets
        const uint64_t rec_bytes_needed = 16 * (max_data + 1) + 8 * (max_data + 1);
        uint8_t *d_rec = static_cast<uint8_t *>(M.dev(Memory::D_REC, rec_bytes_needed));
        if (!d_rec) return finish(ST_E_HIP);
        uint64_t *d_rec_off = reinterpret_cast<uint64_t *>(d_rec);
        x.pass_off = reinterpret_cast<uint64_t *>(d_rec + 8 * (max_data + 1));
        x.pass_len = reinterpret_cast<uint32_t *>(d_rec + 16 * (max_data + 1));
        x.pass_no = x.pass_len + (max_data + 1);
        if (vcfc_line_index_place(d_in, n, n_lines, d_ix1, d_ix2, L, x, s) != hipSuccess ||
            hipMemcpyAsync(hsmall, d_small, 32, hipMemcpyDeviceToHost, s) != hipSuccess || !sync())
            return finish(ST_E_HIP);
        if (hsmall[3]) return finish(ST_E_ARG);
        const uint64_t n_data = hsmall[1], n_pass = hsmall[2];
        // '#' lines: bytes from the host copy, checked in order; the first
        // header line with < 8 terms stops the input there
        std::vector<PassLine> pass;
        int64_t hdr_err = -1;   // chunk line number
        uint64_t hdr_before = 0;
        if (n_pass) {
            pass_off.resize(n_pass); pass_len.resize(n_pass); pass_no.resize(n_pass); pass_before.resize(n_pass);
            if (hipMemcpyAsync(pass_off.data(), x.pass_off, 8 * n_pass, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipMemcpyAsync(pass_len.data(), x.pass_len, 4 * n_pass, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipMemcpyAsync(pass_no.data(), x.pass_no, 4 * n_pass, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipMemcpyAsync(pass_before.data(), x.pass_before, 8 * n_pass, hipMemcpyDeviceToHost, s) != hipSuccess ||
                !sync())
                return finish(ST_E_HIP);
            for (uint64_t k = 0; k < n_pass; k++) {
                const uint8_t *p = h + pass_off[k];
                const uint64_t len = pass_len[k];
                if (!(len >= 2 && p[1] == '#') && !header_ok(p, len)) {
                    hdr_err = pass_no[k];
                    hdr_before = pass_before[k];
                    break;
                }
                PassLine pl;
                pl.before = pass_before[k];
                pl.no = pass_no[k];
                pl.text.assign(p, p + len);
                pl.text.push_back('\n');
                pass.push_back(std::move(pl));
            }
        }
        free_in.put(ch.slot);   // the host copy is no longer needed
        // encode the data lines
        int oslot;
        const double o0 = now_s();
        if (!free_out.get(oslot)) return finish(ST_E_HIP);
        t_wait_out += now_s() - o0;
        OutChunk oc;
        oc.slot = oslot;
        uint64_t good = n_data;   // rows to write
        int st = ST_OK;
        int64_t bad_line = -1;
        uint8_t *d_out = nullptr;
        oc.rec_off.assign(1, 0);
        if (n_data) {
            const VcfcWorkspaceLayout W = vcfc_encode_workspace_layout(n_data, n);
            uint8_t *ws = static_cast<uint8_t *>(M.dev(Memory::D_ENC_WS, W.total));
            const uint64_t cap = vcfc_record_bound(n_data, n) + 64;
            d_out = static_cast<uint8_t *>(M.dev(Memory::D_OUT, cap));
            if (!ws || !d_out) return finish(ST_E_HIP);
            VcfcEncodeArgs a;
            a.buf = d_in; a.line_off = x.line_off; a.line_len = x.line_len; a.n = n_data;
            a.line_bytes_hint = n;
            a.out = d_out; a.out_cap = cap; a.rec_off = d_rec_off;
            vcfc_encode_args_workspace(a, ws, W);
            a.err = d_small + 4;
            a.defer_records = cfg.defer_records ? 1u : 0u;
            oc.rec_off.resize(n_data + 1);
            if (vcfc_encode_device(a, s) != hipSuccess ||
                hipMemcpyAsync(oc.rec_off.data(), d_rec_off, 8 * (n_data + 1), hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipMemcpyAsync(hsmall + 4, d_small + 4, 8, hipMemcpyDeviceToHost, s) != hipSuccess || !sync())
                return finish(ST_E_HIP);
            const uint64_t errw = hsmall[4];
            if (errw != VCFCD_NO_ERROR) {
                good = errw >> 8;
                st = (int)(errw & 0xFF);
                uint32_t ln = 0;
                if (hipMemcpyAsync(&ln, x.line_no + good, 4, hipMemcpyDeviceToHost, s) != hipSuccess || !sync())
                    return finish(ST_E_HIP);
                bad_line = ln;
            }
        }
        // the first failing line of the chunk: a header line or a data line
        bool stop = false;
        if (hdr_err >= 0 && (bad_line < 0 || hdr_err < bad_line)) {
            good = hdr_before;
            st = ST_E_HEADER;
            bad_line = hdr_err;
            stop = true;
        } else if (bad_line >= 0) {
            stop = true;
            while (!pass.empty() && pass.back().before > good) pass.pop_back();   // '#' lines after the failing row
        }
        oc.rec_bytes = oc.rec_off[good];
        if (oc.rec_bytes + 64 > hout_cap[oslot]) {   // pinned output sized by the records actually made
            hout[oslot] = static_cast<uint8_t *>(M.host(Memory::H_OUT0 + oslot, oc.rec_bytes + 64));
            hout_cap[oslot] = hout[oslot] ? oc.rec_bytes + 64 : 0;
            if (!hout[oslot]) return finish(ST_E_HIP);
        }
        oc.data = hout[oslot];
        if (oc.rec_bytes &&
            (hipMemcpyAsync(hout[oslot], d_out, oc.rec_bytes, hipMemcpyDeviceToHost, s) != hipSuccess || !sync()))
            return finish(ST_E_HIP);
        oc.pass = std::move(pass);
        if (oc.pass.empty()) oc.rec_off.clear();
        free_dev.put(ch.dslot);   // its records are on the host
        to_write.put(std::move(oc));
        if (stop) {
            if (err_line) *err_line = (int64_t)(line_base + (uint64_t)bad_line + 1);
            return finish(st);
        }
        line_base += n_lines;
        if (lines_out) *lines_out = line_base;
    }
    return finish(ST_OK);
}

// compress() over VCF file bytes already resident in device memory: d_in[0, N)
// holds the file's bytes as read (N > 0, d_in[N - 1] == '\n'), the .vcfc bytes
// go to d_out[0, *out_len).  The GPU stage of compress_stream without the
// transfer stages: chunks of whole lines (up to cfg.chunk bytes, grown to
// hold a longer line, up to cfg.max_chunk; by default the whole input)
// are line-indexed and encoded in place; a chunk whose '#' lines all precede
// its data lines (every real VCF) is encoded straight behind them into
// d_out, one with interleaved '#' lines through a scratch buffer.  The host
// only reads the index counts, the '#' lines (checked: >= 8 terms, as the
// writer path) and a window before each chunk end.
inline int compress_device(const uint8_t *d_in, uint64_t N, uint8_t *d_out, uint64_t out_cap, uint64_t *out_len,
                           Memory &M, hipStream_t s, const Config &cfg, int64_t *err_line) {
    using namespace detail;
    if (err_line) *err_line = -1;
    *out_len = 0;
    if (N == 0) return ST_OK;
    const bool trace = cfg.trace;
    if (trace) fprintf(stderr, "compress_device: N=%llu chunk=%llu max=%llu\n", (unsigned long long)N,
                       (unsigned long long)cfg.chunk, (unsigned long long)cfg.max_chunk);
    if (cfg.chunk < 16 || cfg.chunk > cfg.max_chunk) return ST_E_ARG;
    uint64_t *hsmall = static_cast<uint64_t *>(M.host(Memory::H_SMALL, 64));
    uint64_t *d_small = static_cast<uint64_t *>(M.dev(Memory::D_SMALL, 64));
    if (!hsmall || !d_small) return ST_E_HIP;
    auto sync = [&]() { return hipStreamSynchronize(s) == hipSuccess; };
    // (every D2H below lands in pinned memory, so the copies of one step
    // queue behind each other and cost one host round trip per sync: a D2H
    // into pageable memory is synchronous, ~20 us of idle GPU each --
    // round 6, profiles/r06/devfile_trace_*.txt)
    auto d2h = [&](void *dst, const void *src, uint64_t k) {
        return hipMemcpyAsync(dst, src, k, hipMemcpyDeviceToHost, s) == hipSuccess;
    };
    // The sample count S from the "#CHROM" line (in the first MiB) lets the
    // line index hop over a data line's genotypes (vcfc_line_index S_hint);
    // a chunk whose hop index the encoder finds wrong (VCFCD_E_NEWLINE) is
    // indexed again from every byte.  cfg.hop_index false
    // (VCFC_LINE_INDEX_SCAN): always every byte.  The file's last byte comes
    // with the first header window (one round trip); the window stays on the
    // host for the '#' lines' check below (h0: d_in[0, h0_len)).
    uint32_t S_hint = 0, len_hint = 0;
    bool learn = false;
    VcfcHopCands cands;
    memset(&cands, 0, sizeof cands);
    const uint8_t *h0 = nullptr;
    uint64_t h0_len = 0;
    {
        uint8_t *lastp = reinterpret_cast<uint8_t *>(hsmall + 7);
        if (!d2h(lastp, d_in + N - 1, 1)) return ST_E_HIP;
        bool checked = false;
        if (cfg.hop_index) {
            // 64 KiB of the file into pinned memory, 1 MiB if the header is longer
            for (uint64_t want = std::min<uint64_t>(N, 64u << 10);;) {
                uint8_t *h = static_cast<uint8_t *>(M.host(Memory::H_IN0, want));
                if (!h) return ST_E_HIP;
                if (!d2h(h, d_in, want) || !sync()) return ST_E_HIP;
                checked = true;
                h0 = h;
                h0_len = want;
                bool more = false;
                S_hint = header_samples(h, want, &more);
                const uint64_t cap = std::min<uint64_t>(N, 1u << 20);
                if (!more || want >= cap) {
                    learn = S_hint && (cfg.hop_learn > 0 || (cfg.hop_learn < 0 && data_lines_irregular(h, want, S_hint)));
                    len_hint = S_hint ? first_data_line_len(h, want) : 0u;
                    if (learn) learn_candidates(h, want, S_hint, &cands);
                    break;
                }
                want = cap;
            }
            if (S_hint < 32) S_hint = 0;   // (the check reads 32 tokens)
        }
        if (!checked && !sync()) return ST_E_HIP;
        if (*lastp != '\n') {
            if (trace) fprintf(stderr, "compress_device: last byte %u\n", *lastp);
            return ST_E_ARG;
        }
        if (trace) fprintf(stderr, "compress_device: S_hint=%u learn=%d\n", S_hint, (int)learn);
    }
    uint64_t pos = 0, o = 0, line_base = 0;
    constexpr uint64_t WIN = 1ull << 16;
    std::vector<uint8_t> win;
    while (pos < N) {
        // ---- the chunk: whole lines [pos, pos + n) ----
        uint64_t lim = cfg.chunk, n = 0;
        for (;;) {
            if (N - pos <= lim) { n = N - pos; break; }
            // the last '\n' of [pos, pos + lim), scanning windows backwards
            uint64_t hi = lim;
            while (hi > 0 && !n) {
                const uint64_t lo = hi > WIN ? hi - WIN : 0;
                win.resize(hi - lo);
                if (!d2h(win.data(), d_in + pos + lo, hi - lo) || !sync()) return ST_E_HIP;
                const void *nl = memrchr(win.data(), '\n', hi - lo);
                if (nl) n = lo + (uint64_t)(static_cast<const uint8_t *>(nl) - win.data()) + 1;
                hi = lo;
            }
            if (n) break;
            if (trace) fprintf(stderr, "compress_device: no line end in [%llu, +%llu)\n", (unsigned long long)pos,
                               (unsigned long long)lim);
            if (lim >= cfg.max_chunk) return ST_E_ARG;   // a line longer than max_chunk
            lim = std::min<uint64_t>(2 * lim, cfg.max_chunk);
        }
        const uint8_t *d_c = d_in + pos;
        if (trace) fprintf(stderr, "compress_device: chunk [%llu, +%llu)\n", (unsigned long long)pos, (unsigned long long)n);
        uint32_t hop = S_hint;
      index_again:
        // ---- line index (as compress_stream; hop: see S_hint) ----
        const VcfcLineIndexLayout L1 = vcfc_line_index_layout(n, 0);
        uint8_t *d_ix1 = static_cast<uint8_t *>(M.dev(Memory::D_IX1, L1.total1));
        if (!d_ix1) return ST_E_HIP;
        VcfcLineIndex x;
        x.counts = d_small;
        if (vcfc_line_index(d_c, n, d_ix1, L1, x, s, hop, cfg.hop_walkers, learn, len_hint, &cands) !=
                hipSuccess ||
            !d2h(hsmall, d_small, 8) || !sync())
            return ST_E_HIP;
        const uint64_t n_lines = hsmall[0];
        // line numbers inside a chunk are 32-bit (k_line_place): a chunk of
        // 2^32 lines or more is refused (a chunk size set on the context
        // splits such an input)
        if (n_lines >= (1ull << 32) - 1) return ST_E_ARG;
        const VcfcLineIndexLayout L = vcfc_line_index_layout(n, n_lines);
        uint8_t *d_ix2 = static_cast<uint8_t *>(M.dev(Memory::D_IX2, L.total2));
        uint8_t *d_lines = static_cast<uint8_t *>(M.dev(Memory::D_LINES, 32 * (n_lines + 1)));
        uint8_t *d_rec = static_cast<uint8_t *>(M.dev(Memory::D_REC, 24 * (n_lines + 1)));
        if (!d_ix2 || !d_lines || !d_rec) return ST_E_HIP;
        uint8_t *q = d_lines;
        x.line_off = reinterpret_cast<uint64_t *>(q); q += 8 * (n_lines + 1);
        x.pass_before = reinterpret_cast<uint64_t *>(q); q += 8 * (n_lines + 1);
        x.line_len = reinterpret_cast<uint32_t *>(q); q += 4 * (n_lines + 1);
        x.line_no = reinterpret_cast<uint32_t *>(q);
        uint64_t *d_rec_off = reinterpret_cast<uint64_t *>(d_rec);
        x.pass_off = reinterpret_cast<uint64_t *>(d_rec + 8 * (n_lines + 1));
        x.pass_len = reinterpret_cast<uint32_t *>(d_rec + 16 * (n_lines + 1));
        x.pass_no = x.pass_len + (n_lines + 1);
        // the counts, and with them the first PK entries of the '#' line
        // arrays (every real header fits): gathered on the device, one D2H
        const uint64_t PK = std::min<uint64_t>(n_lines + 1, 1024);
        uint8_t *hsum = static_cast<uint8_t *>(M.host(Memory::H_IN1, 32 + 24 * PK));
        uint8_t *dsum = static_cast<uint8_t *>(M.dev(Memory::D_IN1, 32 + 24 * PK));
        if (!hsum || !dsum) return ST_E_HIP;
        if (vcfc_line_index_place(d_c, n, n_lines, d_ix1, d_ix2, L, x, s) != hipSuccess ||
            vcfc_index_summary(x, PK, dsum, s) != hipSuccess || !d2h(hsum, dsum, 32 + 24 * PK) || !sync())
            return ST_E_HIP;
        memcpy(hsmall, hsum, 32);
        const uint8_t *hpass = hsum + 32;
        // counts[3]: 1 = a line of 4 GiB or more (k_line_place), 2 = a hop
        // index that missed a line end in a segment of more than NL_SLOT
        // lines (k_nl_place's rescan; the other missed ends reach the encoder
        // inside a data row, VCFCD_E_NEWLINE below).  Either way the scan
        // index decides: it never sets 2, and refuses 1.
        if (hsmall[3]) {
            if (hop) {
                if (cfg.hop_redo) ++*cfg.hop_redo;
                hop = 0;
                goto index_again;
            }
            return ST_E_ARG;
        }
        const uint64_t n_data = hsmall[1], n_pass = hsmall[2];
        // ---- '#' lines: to the host, checked in order ----
        // Each '#' line lies in d_c followed by its '\n' -- exactly the bytes
        // the reference writes (line + "\n") -- so it is placed by a D2D copy;
        // the host only checks the text.  The lines come to the host in one
        // D2H of the span from the first to the last (a real header is one
        // contiguous block), or one D2H per line when the span is much longer
        // than the lines (interleaved '#' lines far apart).
        struct DevPass {
            uint64_t before, off, len;   // data lines before it; offset in d_c, length with the '\n'
            uint32_t no;
        };
        std::vector<DevPass> pass;
        int64_t hdr_err = -1;
        uint64_t hdr_before = 0, pass_bytes = 0;
        bool interleaved = false;
        if (n_pass) {
            std::vector<uint32_t> pl(n_pass), pn(n_pass);
            std::vector<uint64_t> po(n_pass), pb(n_pass);
            if (n_pass <= PK) {
                memcpy(po.data(), hpass, 8 * n_pass);
                memcpy(pb.data(), hpass + 8 * PK, 8 * n_pass);
                memcpy(pl.data(), hpass + 16 * PK, 4 * n_pass);
                memcpy(pn.data(), hpass + 20 * PK, 4 * n_pass);
            } else {
                uint8_t *hp = static_cast<uint8_t *>(M.host(Memory::H_IN1, 24 * n_pass));
                if (!hp || !d2h(hp, x.pass_off, 8 * n_pass) || !d2h(hp + 8 * n_pass, x.pass_before, 8 * n_pass) ||
                    !d2h(hp + 16 * n_pass, x.pass_len, 4 * n_pass) || !d2h(hp + 20 * n_pass, x.pass_no, 4 * n_pass) ||
                    !sync())
                    return ST_E_HIP;
                memcpy(po.data(), hp, 8 * n_pass);
                memcpy(pb.data(), hp + 8 * n_pass, 8 * n_pass);
                memcpy(pl.data(), hp + 16 * n_pass, 4 * n_pass);
                memcpy(pn.data(), hp + 20 * n_pass, 4 * n_pass);
            }
            uint64_t text_bytes = 0;
            for (uint64_t k = 0; k < n_pass; k++) text_bytes += pl[k];
            const uint64_t span = po[n_pass - 1] + pl[n_pass - 1] - po[0];
            const bool one_copy = span <= 2 * text_bytes + (1u << 20);
            // the lines' text: the header window read at the start already
            // holds a header at the file's start (no copy), else pinned D2H
            const uint8_t *text = nullptr;
            std::vector<uint64_t> at(n_pass);   // line k's text at text + at[k]
            if (h0 && pos + po[n_pass - 1] + pl[n_pass - 1] <= h0_len) {
                text = h0 + pos;
                for (uint64_t k = 0; k < n_pass; k++) at[k] = po[k];
            } else {
                uint8_t *tb = static_cast<uint8_t *>(M.host(Memory::H_IN2, std::max<uint64_t>(one_copy ? span : text_bytes, 1)));
                if (!tb) return ST_E_HIP;
                if (one_copy) {
                    if (span && !d2h(tb, d_c + po[0], span)) return ST_E_HIP;
                    for (uint64_t k = 0; k < n_pass; k++) at[k] = po[k] - po[0];
                } else {
                    uint64_t t = 0;
                    for (uint64_t k = 0; k < n_pass; k++) {
                        at[k] = t;
                        if (pl[k] && !d2h(tb + t, d_c + po[k], pl[k])) return ST_E_HIP;
                        t += pl[k];
                    }
                }
                if (!sync()) return ST_E_HIP;
                text = tb;
            }
            for (uint64_t k = 0; k < n_pass; k++) {
                const uint8_t *tx = text + at[k];
                const uint64_t len = pl[k];
                if (!(len >= 2 && tx[1] == '#') && !header_ok(tx, len)) {
                    hdr_err = pn[k];
                    hdr_before = pb[k];
                    break;
                }
                pass.push_back(DevPass{pb[k], po[k], len + 1, pn[k]});
            }
            for (const DevPass &p : pass) {
                pass_bytes += p.len;
                interleaved = interleaved || p.before != 0;
            }
        }
        // ---- encode the data lines: straight into d_out behind the '#'
        // lines, or (interleaved) into a scratch buffer ----
        uint64_t good = n_data;
        int st = ST_OK;
        int64_t bad_line = -1;
        uint8_t *d_recs = nullptr;
        // record offsets: only the few the placement needs come to the host
        // (the batch's total with the encode's error word, the others one
        // round trip each -- only interleaved '#' lines need them)
        auto rec_at = [&](uint64_t k, uint64_t *v) {
            *v = 0;
            if (!n_data || k == 0) return true;
            if (k == n_data) { *v = hsmall[5]; return true; }
            return d2h(hsmall + 6, d_rec_off + k, 8) && sync() && (*v = hsmall[6], true);
        };
        // '#' lines that all precede the chunk's data lines (every real VCF):
        // their D2D copies go ahead of the encode, so the encode's one
        // round trip covers them (they land at d_out[o, o + pass_bytes)
        // whatever the encode finds: none follows a data row)
        bool pass_placed = false;
        if (!interleaved && !pass.empty()) {
            if (o + pass_bytes > out_cap) return ST_E_NOSPACE;
            uint64_t q = o, rs = pass[0].off, rl = 0, rd = o;
            for (const DevPass &p : pass) {
                if (rl && rs + rl != p.off) {
                    if (hipMemcpyAsync(d_out + rd, d_c + rs, rl, hipMemcpyDeviceToDevice, s) != hipSuccess) return ST_E_HIP;
                    rs = p.off;
                    rd = q;
                    rl = 0;
                }
                rl += p.len;
                q += p.len;
            }
            if (rl && hipMemcpyAsync(d_out + rd, d_c + rs, rl, hipMemcpyDeviceToDevice, s) != hipSuccess) return ST_E_HIP;
            pass_placed = true;
        }
        if (n_data) {
            const VcfcWorkspaceLayout W = vcfc_encode_workspace_layout(n_data, n);
            uint8_t *ws = static_cast<uint8_t *>(M.dev(Memory::D_ENC_WS, W.total));
            uint64_t cap;
            if (interleaved) {
                cap = vcfc_record_bound(n_data, n) + 64;
                d_recs = static_cast<uint8_t *>(M.dev(Memory::D_OUT, cap));
            } else {
                if (o + pass_bytes > out_cap) return ST_E_NOSPACE;
                d_recs = d_out + o + pass_bytes;
                cap = out_cap - o - pass_bytes;
            }
            if (!ws || !d_recs) return ST_E_HIP;
            VcfcEncodeArgs a;
            a.buf = d_c; a.line_off = x.line_off; a.line_len = x.line_len; a.n = n_data;
            a.line_bytes_hint = n;
            a.out = d_recs; a.out_cap = cap; a.rec_off = d_rec_off;
            vcfc_encode_args_workspace(a, ws, W);
            a.err = d_small + 4;
            a.nl_check = hop != 0;
            a.defer_records = cfg.defer_records ? 1u : 0u;
            if (vcfc_encode_device(a, s) != hipSuccess || !d2h(hsmall + 4, d_small + 4, 8) ||
                !d2h(hsmall + 5, d_rec_off + n_data, 8) || !sync())
                return ST_E_HIP;
            const uint64_t errw = hsmall[4];
            if (errw != VCFCD_NO_ERROR && (errw & 0xFF) == VCFCD_E_NEWLINE) {
                if (trace) fprintf(stderr, "compress_device: hop index missed a line end (row %llu)\n",
                                   (unsigned long long)(errw >> 8));
                if (cfg.hop_redo) ++*cfg.hop_redo;
                hop = 0;
                goto index_again;
            }
            if (errw != VCFCD_NO_ERROR) {
                good = errw >> 8;
                st = (int)(errw & 0xFF);
                if (st == ST_E_NOSPACE) return ST_E_NOSPACE;
                uint32_t ln = 0;
                if (!d2h(&ln, x.line_no + good, 4) || !sync()) return ST_E_HIP;
                bad_line = ln;
            }
        }
        bool stop = false;
        if (hdr_err >= 0 && (bad_line < 0 || hdr_err < bad_line)) {
            good = hdr_before;
            st = ST_E_HEADER;
            bad_line = hdr_err;
            stop = true;
        } else if (bad_line >= 0) {
            stop = true;
            while (!pass.empty() && pass.back().before > good) pass.pop_back();   // '#' lines after the failing row
        }
        // ---- place the '#' lines (and, interleaved, the record runs); runs
        // of '#' lines adjacent in the input and in the output are one copy ----
        uint64_t at = 0;   // records placed so far
        uint64_t run_src = 0, run_dst = 0, run_len = 0;
        auto flush_run = [&]() {
            const bool ok = !run_len ||
                            hipMemcpyAsync(d_out + run_dst, d_c + run_src, run_len, hipMemcpyDeviceToDevice, s) == hipSuccess;
            run_len = 0;
            return ok;
        };
        if (pass_placed) {   // (copied ahead of the encode)
            o += pass_bytes;
            pass.clear();
        }
        for (const DevPass &p : pass) {
            uint64_t upto;
            if (!rec_at(std::min<uint64_t>(p.before, good), &upto)) return ST_E_HIP;
            if (upto > at) {
                if (!flush_run()) return ST_E_HIP;
                if (o + upto - at > out_cap) return ST_E_NOSPACE;
                if (interleaved && hipMemcpyAsync(d_out + o, d_recs + at, upto - at, hipMemcpyDeviceToDevice, s) != hipSuccess)
                    return ST_E_HIP;
                o += upto - at;
                at = upto;
            }
            if (o + p.len > out_cap) return ST_E_NOSPACE;
            if (run_len && (run_src + run_len != p.off || run_dst + run_len != o) && !flush_run()) return ST_E_HIP;
            if (!run_len) { run_src = p.off; run_dst = o; }
            run_len += p.len;
            o += p.len;
        }
        if (!flush_run()) return ST_E_HIP;
        uint64_t rec_end;
        if (!rec_at(good, &rec_end)) return ST_E_HIP;
        if (rec_end > at) {
            if (o + rec_end - at > out_cap) return ST_E_NOSPACE;
            if (interleaved && hipMemcpyAsync(d_out + o, d_recs + at, rec_end - at, hipMemcpyDeviceToDevice, s) != hipSuccess)
                return ST_E_HIP;
            o += rec_end - at;
        }
        if (!sync()) return ST_E_HIP;
        *out_len = o;
        if (stop) {
            if (err_line) *err_line = (int64_t)(line_base + (uint64_t)bad_line + 1);
            return st;
        }
        line_base += n_lines;
        pos += n;
    }
    return ST_OK;
}

}  // namespace vcfc_ing
