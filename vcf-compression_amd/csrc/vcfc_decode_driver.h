// vcfc_decode_driver.h -- host driver of the GPU decoder,
// shared by the C ABI (vcfc_api.cpp) and the CPU emulator harness
// (tests/simt_emu/emu_api.cpp), so the same control flow is tested on both.
//
// It mirrors decompress2_fd's data-line loop (reference
// src/compress.cpp:1214-1257 + decompress2_data_line :741-986):
//   1. hop the LEN headers on the host to find record starts;
//   2. plan every record on the GPU (line sizes, statuses, first failure);
//   3. write the lines before the first failure in output batches;
//   4. where a record's byte-serial parse ends off its LEN hop, or hopping
//      stopped early, decode the rest the reference's way (k_dec_stream);
//   5. VCFC_E_FORMAT where the reference throws, after sinking every line
//      the reference would have written first.
#pragma once
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <functional>
#include <thread>
#include <vector>

#include "vcfc_device.h"
#include "vcfc_queue.h"

namespace vcfc_dec {

constexpr int ST_OK = 0, ST_E_HIP = 6, ST_E_IO = 7, ST_E_FORMAT = 8;   // = include/vcfc.h codes

// Device buffers, owned by the caller (one slot each; contents not kept).
struct Buffers {
    virtual ~Buffers() {}
    enum { IN = 0, REC, WS, OUT, LINE_OFF, SMALL, FLAG, QREF, N_SLOTS };
    virtual void *get(int slot, uint64_t bytes) = 0;   // nullptr on failure
    // host staging (pinned where the implementation can): HOST_OUT receives
    // decoded lines (D2H), HOST_IN assembles uploads; contents not kept
    enum { HOST_OUT = 0, HOST_IN, HOST_IN2, N_HOST };
    virtual uint8_t *host(int slot, uint64_t bytes) {
        if (hv[slot].size() < bytes || hv[slot].empty()) hv[slot].resize(bytes < 64 ? 64 : bytes);
        return hv[slot].data();
    }
    std::vector<uint8_t> hv[N_HOST];
};

// Appends decoded bytes (host memory); false aborts with ST_E_IO.
using Sink = std::function<bool(const uint8_t *, uint64_t)>;

// Metadata + header lines of a .vcfc (decompress2_metadata_headers[_fd],
// reference src/compress.cpp:995-1211): '##' lines then one '#' line, each
// '\n'-terminated; sample_count = TABs after the 8th on the header line.  A
// file with no data lines is an error there (the stale first byte '#' after
// EOF reads as a header row after the header).
inline int parse_header(const uint8_t *in, uint64_t n, uint64_t *data_off, uint64_t *sample_count) {
    bool got_meta = false, got_header = false;
    uint64_t ip = 0, samples = 0;
    for (;;) {
        if (ip >= n) return ST_E_FORMAT;
        const uint8_t c1 = in[ip];
        if (c1 != '#') {
            if (!got_meta || !got_header) return ST_E_FORMAT;
            break;
        }
        if (got_header) return ST_E_FORMAT;
        if (ip + 1 >= n) return ST_E_FORMAT;
        const uint8_t c2 = in[ip + 1];
        if (c2 == '#') got_meta = true;
        else { if (!got_meta) return ST_E_FORMAT; got_header = true; }
        uint64_t q = ip + 2, tabs = 0;
        for (;;) {
            if (q >= n) return ST_E_FORMAT;
            const uint8_t c3 = in[q++];
            if (c3 == '\n') break;
            if (got_header && c3 == '\t' && ++tabs > 8) samples++;
        }
        ip = q;
    }
    *data_off = ip;
    if (sample_count) *sample_count = samples;
    return ST_OK;
}

// Record starts by LEN hops from 0 (read_compressed_line_length_headers,
// compress.cpp:270-331): records lying wholly inside [0, n) whose two
// headers carry extension bits 11 (utils.hpp:198-206) and LEN >= 4.
// rec.back() = where hopping stopped (n, or a record the byte-serial path
// must look at: short tail, bad header bits, LEN past the end).
inline void hop(const uint8_t *in, uint64_t n, std::vector<uint64_t> &rec) {
    rec.clear();
    uint64_t p = 0;
    while (n - p >= 8) {
        const uint8_t *h = in + p;
        if ((h[0] >> 6) != 3u || (h[4] >> 6) != 3u) break;
        const uint64_t L = ((uint64_t)(h[0] & 0x3Fu) << 24) | ((uint64_t)h[1] << 16) | ((uint64_t)h[2] << 8) | h[3];
        if (L < 4 || L + 4 > n - p) break;
        rec.push_back(p);
        p += 4 + L;
    }
    rec.push_back(p);
}

// Decode the records [rec[i], rec[i + 1]), i < nrec, of the uploaded data
// section d_in[0, n) (d_rec: the same offsets on the device), sinking their
// lines in order; d_select (device, nullable): records with select[i] == 0
// get no line.  Stops early at the first record the reference would not
// leave at its end: *stop = 1 where it throws (lines before it sunk), 2 where
// its parse ends off the record end, at *cont (its line sunk).  *stop = 0:
// all records decoded.  line_end (optional): the end of every sunk line,
// counted from the first byte this call sinks.
inline int decode_records(const uint8_t *d_in, uint64_t n, uint64_t S, const uint64_t *d_rec, const uint8_t *d_select,
                          uint64_t nrec, Buffers &B, hipStream_t s, const Sink &sink, uint64_t out_batch, int *stop,
                          uint64_t *cont, std::vector<uint64_t> *line_end = nullptr) {
    *stop = 0;
    if (!nrec) return ST_OK;
    const VcfcDecodeLayout L = vcfc_decode_workspace_layout(nrec);
    uint8_t *ws = static_cast<uint8_t *>(B.get(Buffers::WS, L.total));
    uint64_t *d_loff = static_cast<uint64_t *>(B.get(Buffers::LINE_OFF, 8 * (nrec + 1)));
    if (!ws || !d_loff) return ST_E_HIP;
    VcfcDecodeArgs a;
    a.in = d_in; a.n_bytes = n; a.rec_start = d_rec; a.select = d_select; a.n = nrec; a.S = S;
    a.out = nullptr; a.out_cap = 0; a.line_off = d_loff;
    a.st = reinterpret_cast<uint32_t *>(ws + L.st);
    a.line_size = reinterpret_cast<uint32_t *>(ws + L.line_size);
    a.end = reinterpret_cast<uint64_t *>(ws + L.end);
    a.seq_list = reinterpret_cast<uint32_t *>(ws + L.seq_list);
    a.seq_count = reinterpret_cast<uint32_t *>(ws + L.seq_count);
    a.err = reinterpret_cast<uint64_t *>(ws + L.err);
    a.partials = reinterpret_cast<uint64_t *>(ws + L.partials);
    // plan (light first: header + REQ only), then write in output batches;
    // a batch whose write finds a record the light plan got wrong is
    // re-planned exactly (lines already sunk keep their bytes: every line
    // before the first wrong record had the right size)
    bool exact = false;
    uint64_t n_lines = 0;
    std::vector<uint64_t> loff;
    auto plan = [&]() -> int {
        if (vcfc_decode_plan(a, exact, s) != hipSuccess) return ST_E_HIP;
        uint64_t err = 0;
        if (hipMemcpyAsync(&err, a.err, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            return ST_E_HIP;
        n_lines = nrec;
        *stop = 0;
        if (err != VCFCD_NO_ERROR) {
            const uint64_t k = err >> 8;
            if ((err & 0xFF) == 2) {   // parse of record k ends off its end: keep its line, continue there
                n_lines = k + 1;
                *stop = 2;
                if (hipMemcpyAsync(cont, a.end + k, 8, hipMemcpyDeviceToHost, s) != hipSuccess) return ST_E_HIP;
            } else {
                n_lines = k;
                *stop = 1;
            }
        }
        loff.resize(n_lines + 1);
        if (hipMemcpyAsync(loff.data(), d_loff, 8 * (n_lines + 1), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return ST_E_HIP;
        return ST_OK;
    };
    int pst = plan();
    if (pst) return pst;
    for (uint64_t i0 = 0; i0 < n_lines;) {
        uint64_t i1 = i0 + 1;
        while (i1 < n_lines && loff[i1 + 1] - loff[i0] <= out_batch) i1++;
        const uint64_t bytes = loff[i1] - loff[i0];
        uint8_t *d_out = static_cast<uint8_t *>(B.get(Buffers::OUT, bytes + 64));
        if (!d_out) return ST_E_HIP;
        a.out = d_out - loff[i0];   // lines are written at out + line_off[i]
        a.out_cap = loff[i1];
        uint64_t err = 0;
        if (vcfc_decode_write(a, i0, i1, s) != hipSuccess || hipMemcpyAsync(&err, a.err, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return ST_E_HIP;
        if (err != VCFCD_NO_ERROR && (err & 0xFF) == 4 && !exact) {
            exact = true;
            if ((pst = plan())) return pst;
            continue;   // same i0, exact sizes
        }
        uint8_t *host = B.host(Buffers::HOST_OUT, bytes + 64);
        if (!host) return ST_E_HIP;
        if (hipMemcpyAsync(host, d_out, bytes, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            return ST_E_HIP;
        if (!sink(host, bytes)) return ST_E_IO;
        if (line_end)
            for (uint64_t i = i0; i < i1; i++) line_end->push_back(loff[i + 1] - loff[0]);
        i0 = i1;
    }
    return ST_OK;
}

// Run a one-lane byte-serial kernel (count pass, then write pass) and sink
// its output.  run(out, st) enqueues it; st[0] = 2 means the reference throws.
template <class Run>
inline int stream_tail(Buffers &B, hipStream_t s, const Sink &sink, Run &&run) {
    uint64_t *d_small = static_cast<uint64_t *>(B.get(Buffers::SMALL, 64));
    if (!d_small) return ST_E_HIP;
    uint64_t st[3] = {0, 0, 0};
    if (run(nullptr, d_small) != hipSuccess || hipMemcpyAsync(st, d_small, 24, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return ST_E_HIP;
    if (st[1]) {
        uint8_t *d_out = static_cast<uint8_t *>(B.get(Buffers::OUT, st[1] + 64));
        if (!d_out) return ST_E_HIP;
        std::vector<uint8_t> host(st[1]);
        if (run(d_out, d_small) != hipSuccess || hipMemcpyAsync(host.data(), d_out, st[1], hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return ST_E_HIP;
        if (!sink(host.data(), st[1])) return ST_E_IO;
    }
    return st[0] == 2 ? ST_E_FORMAT : ST_OK;
}

inline uint8_t *upload(Buffers &B, int slot, const uint8_t *h, uint64_t n, hipStream_t s) {
    uint8_t *d = static_cast<uint8_t *>(B.get(slot, n + 64));
    if (d && n && hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s) != hipSuccess) return nullptr;
    return d;
}

// Decode a .vcfc data section (host bytes h_in[0, n); uploaded here).
inline int decode_section(const uint8_t *h_in, uint64_t n, uint64_t S, Buffers &B, hipStream_t s, const Sink &sink,
                          uint64_t out_batch = 1ull << 30) {
    std::vector<uint64_t> rec;
    hop(h_in, n, rec);
    const uint8_t *d_in = upload(B, Buffers::IN, h_in, n, s);
    const uint64_t *d_rec = reinterpret_cast<const uint64_t *>(
        upload(B, Buffers::REC, reinterpret_cast<const uint8_t *>(rec.data()), 8 * rec.size(), s));
    if (!d_in || !d_rec) return ST_E_HIP;
    int stop = 0;
    uint64_t p_stream = rec.back();   // byte-serial continuation point
    int st = decode_records(d_in, n, S, d_rec, nullptr, rec.size() - 1, B, s, sink, out_batch, &stop, &p_stream);
    if (st) return st;
    if (stop == 1) return ST_E_FORMAT;
    if (n - p_stream < 8) return ST_OK;   // clean end (:768-774)
    return stream_tail(B, s, sink, [&](uint8_t *out, uint64_t *dst) { return vcfc_decode_stream(d_in, n, p_stream, S, ~0ull, out, dst, s); });
}

// Range query over a .vcfc data section (query_compressed_file, reference
// src/main.cpp:3777-3929): the matching lines, no header.
//   1. hop the LEN headers; one lane per record finds CHROM/POS and the
//      match flag (k_query_match);
//   2. the records before the first irregular one decode through
//      decode_records, the flags selecting the matching ones;
//   3. from the first record where the reference's walk leaves the hops (a
//      CHROM/POS past the record, a matching record whose parse ends off
//      its hop, the hop end), k_query_stream walks the rest byte-serially.
inline int query_section(const uint8_t *h_in, uint64_t n, uint64_t S, const uint8_t *qref, uint64_t qref_len,
                         int has_range, uint64_t qstart, uint64_t qend, Buffers &B, hipStream_t s, const Sink &sink,
                         uint64_t out_batch = 1ull << 30) {
    if (qref_len > 0xFFFFFFFFull) return ST_E_FORMAT;
    std::vector<uint64_t> rec;
    hop(h_in, n, rec);
    const uint64_t nrec = rec.size() - 1;
    const uint8_t *d_in = upload(B, Buffers::IN, h_in, n, s);
    const uint8_t *d_ref = upload(B, Buffers::QREF, qref, qref_len, s);
    uint64_t *d_small = static_cast<uint64_t *>(B.get(Buffers::SMALL, 64));
    if (!d_in || !d_ref || !d_small) return ST_E_HIP;
    VcfcQuery q;
    q.ref = d_ref; q.ref_len = (uint32_t)qref_len; q.has_range = has_range ? 1u : 0u; q.start = qstart; q.end = qend;
    uint64_t p_stream = rec.back();
    if (nrec) {
        const uint64_t *d_rec = reinterpret_cast<const uint64_t *>(
            upload(B, Buffers::REC, reinterpret_cast<const uint8_t *>(rec.data()), 8 * (nrec + 1), s));
        uint8_t *d_flag = static_cast<uint8_t *>(B.get(Buffers::FLAG, nrec + 64));
        if (!d_rec || !d_flag) return ST_E_HIP;
        uint64_t err = 0;
        if (vcfc_query_match(d_in, d_rec, nrec, q, d_flag, d_small, s) != hipSuccess ||
            hipMemcpyAsync(&err, d_small, 8, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            return ST_E_HIP;
        // records before the first irregular one k: the matching ones decode
        const uint64_t k = err == VCFCD_NO_ERROR ? nrec : err >> 8;
        int stop = 0;
        uint64_t cont = 0;
        int st = decode_records(d_in, n, S, d_rec, d_flag, k, B, s, sink, out_batch, &stop, &cont);
        if (st) return st;
        if (stop == 1) return ST_E_FORMAT;
        if (stop == 2) p_stream = cont;
        else if (k < nrec) {
            if ((err & 0xFF) == 2) return ST_E_FORMAT;   // POS of record k does not parse
            p_stream = rec[k];
        }
    }
    if (p_stream >= n) return ST_OK;
    return stream_tail(B, s, sink, [&](uint8_t *out, uint64_t *dst) { return vcfc_query_stream(d_in, n, p_stream, S, q, out, dst, s); });
}


// ---------------------------------------------------------------------------
// Sparse-file query: query_sparse_file_fd, reference
// src/main.cpp:235-582, over a file written by sparsify (record i at
// data_start + (3e8 + POS_i) * 16384 behind BE dist_to_prev / dist_to_next).
// The walk is host I/O with the reference's own lseek/read sequence (header,
// single-slot lookup or SEEK_DATA + slot alignment + hole skipping, then the
// dist_to_next hops).  The lines are decoded on the GPU: the walk runs ahead
// in geometrically growing batches of records, each batch decodes in one
// decode_records call, and the reference's per-line verdicts (CHROM/POS of
// the decoded line, end of range, end of reference) are then applied in
// order.  A line whose parse leaves its record (the reference reads on into
// the hole or the next record) is decoded again from a window of the file
// (k_dec_stream, one line), grown until the parse ends inside it.
struct SparseQuery {
    const uint8_t *ref;
    uint64_t ref_len;
    int has_range;
    uint64_t start, end;
};

constexpr int64_t SQ_STRIDE = 4 * 4096;   // multiplication_factor * block_size (src/sparse.hpp:29-32)

inline uint64_t sq_be64(const uint8_t *b) {
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = (v << 8) | b[i];
    return v;
}
// compute_sparse_offset (src/sparse.cpp:18-51; the name is ignored)
inline uint64_t sq_slot(uint64_t pos) { return (300000000ull + pos) * (uint64_t)SQ_STRIDE; }

// bytes read at off (short only at EOF); -1 on a read error
inline int64_t sq_pread(int fd, uint8_t *b, uint64_t k, uint64_t off) {
    uint64_t got = 0;
    while (got < k) {
        const ssize_t r = pread(fd, b + got, std::min<uint64_t>(k - got, 1ull << 30), (off_t)(off + got));
        if (r < 0) return -1;
        if (r == 0) break;
        got += (uint64_t)r;
    }
    return (int64_t)got;
}

// strtoul(s, &end, 10) with end == s + n required; "" is 0 (main.cpp:520-524)
inline bool sq_strtoul_whole(const uint8_t *s, uint64_t n, uint64_t *out) {
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
        ovf = ovf || v > (~0ull - d) / 10;
        v = v * 10 + d;
    }
    if (i != n) return false;
    *out = ovf ? ~0ull : (neg ? 0ull - v : v);
    return true;
}

// One line the reference's way from file offset p
// (decompress2_data_line_FILEwrapper, src/compress.cpp:483-739), on the GPU
// over a window of the file grown x4 until the parse ends inside it or the
// window reaches EOF (1 GiB at most).  Appends the line, sets *end.
inline int sq_line_window(int fd, uint64_t fsize, uint64_t p, uint64_t S, Buffers &B, hipStream_t s,
                          std::vector<uint8_t> &line, uint64_t *end) {
    std::vector<uint8_t> win;
    for (uint64_t w = 1ull << 16;; w *= 4) {
        const uint64_t avail = p < fsize ? fsize - p : 0;
        const uint64_t n = std::min(w, avail);
        win.resize(n);
        const int64_t got = sq_pread(fd, win.data(), n, p);
        if (got < 0) return ST_E_IO;
        const uint8_t *d_win = upload(B, Buffers::FLAG, win.data(), (uint64_t)got, s);
        uint64_t *d_small = static_cast<uint64_t *>(B.get(Buffers::SMALL, 64));
        if (!d_win || !d_small) return ST_E_HIP;
        uint64_t st[4] = {0, 0, 0, 0};
        if (vcfc_decode_stream(d_win, (uint64_t)got, 0, S, 1, nullptr, d_small, s) != hipSuccess ||
            hipMemcpyAsync(st, d_small, 32, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            return ST_E_HIP;
        if (st[2] == 1) {
            uint8_t *d_out = static_cast<uint8_t *>(B.get(Buffers::OUT, st[1] + 64));
            if (!d_out) return ST_E_HIP;
            const uint64_t o = line.size();
            line.resize(o + st[1]);
            if (vcfc_decode_stream(d_win, (uint64_t)got, 0, S, 1, d_out, d_small, s) != hipSuccess ||
                hipMemcpyAsync(line.data() + o, d_out, st[1], hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                return ST_E_HIP;
            *end = p + st[3];
            return ST_OK;
        }
        // EOF at the line start (status 0) and a failed parse both throw (main.cpp:324-328, 482-486)
        if ((uint64_t)got == avail || w >= (1ull << 30)) return ST_E_FORMAT;
    }
}

// the walk's view of one record
struct SqRec {
    uint64_t ls;      // line_start_offset: its 16 distance bytes
    uint64_t dnext;   // dist_to_next (0: end of reference)
    int walk;         // 0, or ST_E_FORMAT: the reference throws reading its distances
    bool sync;        // the hop's lseek fails: the next read starts where this line's parse ends
    uint64_t pre, npre;   // the first bytes from ls, read with the distances: pre[pre, + npre)
};
constexpr uint64_t SQ_PRE = 1024;   // bytes read per hop (holds most records whole)

// The largest offset lseek(SEEK_SET) accepts on this file (validity is
// monotonic: 0 <= x <= the filesystem's maximum file size), by bisection.
inline int64_t sq_max_seek(int fd) {
    int64_t lo = 0, hi = INT64_MAX;
    if (lseek(fd, (off_t)hi, SEEK_SET) == (off_t)hi) return hi;
    while (hi - lo > 1) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (lseek(fd, (off_t)mid, SEEK_SET) == (off_t)mid) lo = mid;
        else hi = mid;
    }
    return lo;
}

// Walk up to `want` records from ls (linear traversal, main.cpp:436-566):
// stops after an end-of-reference record, a walk error, or a failing hop.
inline int sq_walk(int fd, uint64_t ls, uint64_t want, int64_t max_seek, std::vector<SqRec> &recs,
                   std::vector<uint8_t> &pre) {
    recs.clear();
    pre.clear();
    while (recs.size() < want) {
        const uint64_t o = pre.size();
        pre.resize(o + SQ_PRE);
        const int64_t k = sq_pread(fd, pre.data() + o, SQ_PRE, ls);
        if (k < 0) return ST_E_IO;
        pre.resize(o + (uint64_t)k);
        uint8_t h[16] = {0};
        memcpy(h, pre.data() + o, std::min<uint64_t>(16, (uint64_t)k));
        SqRec r;
        r.ls = ls; r.dnext = sq_be64(h + 8); r.walk = 0; r.sync = false; r.pre = o; r.npre = (uint64_t)k;
        if (k < 16) { r.walk = ST_E_FORMAT; recs.push_back(r); break; }                  // :454-456
        if (sq_be64(h) == 0 && r.dnext == 0) { r.walk = ST_E_FORMAT; recs.push_back(r); break; }   // :464-466
        const int64_t next = (int64_t)(ls + r.dnext);   // lseek64(dnext - bytes read, SEEK_CUR) lands here
        if (r.dnext && (next < 0 || next > max_seek)) r.sync = true;
        recs.push_back(r);
        if (r.dnext == 0 || r.sync) break;
        ls = (uint64_t)next;
    }
    return ST_OK;
}

// One batch of the walk: the records, the bytes read with their distances,
// and the regular records (sane header, whole in the file) staged back to back
// in a pinned upload buffer.
struct SqBatch {
    std::vector<SqRec> recs;
    std::vector<uint8_t> pre;
    std::vector<uint64_t> roff, reg;   // staging offsets (+ end) and record index of the regular records
    uint64_t hbytes = 0;
    int slot = 0;                      // Buffers::HOST_IN / HOST_IN2
    int st = ST_OK;                    // walk I/O error
    bool last = false;                 // the walker stops after this batch
};

inline int sq_stage(int fd, SqBatch &b, Buffers &B) {
    b.roff.clear();
    b.reg.clear();
    std::vector<uint64_t> rlen;
    uint64_t hbytes = 0;
    for (uint64_t i = 0; i < b.recs.size(); i++) {
        const SqRec &r = b.recs[i];
        if (r.walk) break;
        if (r.npre < 24) continue;
        const uint8_t *h8 = b.pre.data() + r.pre + 16;
        if ((h8[0] >> 6) != 3u || (h8[4] >> 6) != 3u) continue;
        const uint64_t L = ((uint64_t)(h8[0] & 0x3Fu) << 24) | ((uint64_t)h8[1] << 16) | ((uint64_t)h8[2] << 8) | h8[3];
        if (L < 4) continue;
        b.roff.push_back(hbytes);
        rlen.push_back(4 + L);
        b.reg.push_back(i);
        hbytes += 4 + L;
    }
    uint8_t *hbuf = B.host(b.slot == 0 ? Buffers::HOST_IN : Buffers::HOST_IN2, hbytes + 64);
    if (!hbuf) return ST_E_HIP;
    uint64_t w = 0, q = 0;
    for (uint64_t j = 0; j < b.reg.size(); j++) {
        const SqRec &r = b.recs[b.reg[j]];
        const uint64_t k = rlen[j];
        if (16 + k <= r.npre) {
            memcpy(hbuf + w, b.pre.data() + r.pre + 16, k);
        } else {
            const int64_t got = sq_pread(fd, hbuf + w, k, r.ls + 16);
            if (got < 0) return ST_E_IO;
            if (got != (int64_t)k) continue;   // short (EOF): the window path decides
        }
        b.roff[q] = w;
        b.reg[q] = b.reg[j];
        q++;
        w += k;
    }
    b.roff.resize(q);
    b.reg.resize(q);
    b.roff.push_back(w);
    b.hbytes = w;
    return ST_OK;
}

// Linear traversal (main.cpp:436-566) from line_start_offset ls as a
// pipeline: a walker thread reads batches of records ahead (32 records,
// growing to 4 096) into two pinned staging buffers; this thread decodes each
// batch on the GPU and applies the reference's verdicts line by line; a
// writer thread writes the accepted lines (two line buffers).  The walk may
// run up to two batches past the reference's last record; nothing it reads
// there is used.
inline int sq_traverse(int fd, uint64_t fsize, uint64_t ls, uint64_t S, const SparseQuery &q, Buffers &B,
                       hipStream_t s, const Sink &sink, bool trace) {
    const int64_t max_seek = sq_max_seek(fd);
    constexpr uint64_t SQ_BATCH = 4096;
    struct Trace {   // stage times (VCFC_TRACE_SPARSE_QUERY prints them to stderr)
        bool on = false;
        double walk = 0, dec = 0, eval = 0, wait_w = 0, wait_out = 0, total = 0;
        uint64_t recs = 0, batches = 0;
        static double now() {
            return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
        }
        ~Trace() {
            if (on)
                fprintf(stderr, "sparse_query: %llu records in %llu batches, %.1f ms: walk+stage %.1f ms (walker "
                                "thread), GPU decode %.1f ms, verdicts %.1f ms, waiting for the walker %.1f ms, "
                                "for a line buffer %.1f ms\n", (unsigned long long)recs, (unsigned long long)batches,
                        total * 1e3, walk * 1e3, dec * 1e3, eval * 1e3, wait_w * 1e3, wait_out * 1e3);
        }
    } tr;
    tr.on = trace;
    const double t_begin = Trace::now();
    // ---- writer ------------------------------------------------------------
    struct WriteJob {
        int buf = 0;
        std::vector<std::pair<uint64_t, uint64_t>> spans;
    };
    std::vector<uint8_t> lines[2];
    vcfc_q::Queue<WriteJob> jobs;
    vcfc_q::Queue<int> free_lines;
    free_lines.put(0);
    free_lines.put(1);
    std::atomic<bool> write_failed{false};
    std::thread writer([&] {
        WriteJob j;
        while (jobs.get(j)) {
            for (const auto &sp : j.spans)
                if (!write_failed && !sink(lines[j.buf].data() + sp.first, sp.second - sp.first)) write_failed = true;
            free_lines.put(j.buf);
        }
    });
    int status = ST_OK;
    for (bool more = true; more;) {
        // ---- walker (from ls) --------------------------------------------------
        vcfc_q::Queue<SqBatch> batches;
        vcfc_q::Queue<int> free_slots;
        free_slots.put(0);
        free_slots.put(1);
        std::atomic<bool> stop{false};
        double walk_t = 0;
        std::thread walker([&, ls] {
            uint64_t at = ls;
            for (uint64_t want = 32;; want = std::min<uint64_t>(want * 4, SQ_BATCH)) {
                int slot;
                if (stop || !free_slots.get(slot)) break;
                const double t0 = Trace::now();
                SqBatch b;
                b.slot = slot;
                b.st = sq_walk(fd, at, want, max_seek, b.recs, b.pre);
                if (!b.st) b.st = sq_stage(fd, b, B);
                const SqRec *e = b.recs.empty() ? nullptr : &b.recs.back();
                b.last = b.st || !e || e->walk || e->dnext == 0 || e->sync;
                if (!b.last) at = e->ls + e->dnext;
                walk_t += Trace::now() - t0;
                const bool last = b.last;
                batches.put(std::move(b));
                if (last) break;
            }
            batches.close();
        });
        // ---- GPU decode + verdicts (this thread) ---------------------------------
        auto finish_walker = [&] {
            stop = true;
            free_slots.close();
            walker.join();
        };
        SqBatch b;
        bool resume = false;   // the walk continues after a sync record's parse end
        for (;;) {
            double t0 = Trace::now();
            if (!batches.get(b)) { more = false; break; }   // (the walker always ends with a last batch)
            tr.wait_w += Trace::now() - t0;
            if (b.st) { status = b.st; more = false; break; }
            const uint64_t nr = b.recs.size();
            tr.recs += nr;
            tr.batches++;
            int lb;
            t0 = Trace::now();
            if (!free_lines.get(lb)) { status = ST_E_IO; more = false; break; }
            tr.wait_out += Trace::now() - t0;
            std::vector<uint8_t> &L = lines[lb];
            L.clear();
            std::vector<uint64_t> lo(nr, ~0ull), le(nr, 0), pend(nr, 0);
            t0 = Trace::now();
            const uint64_t nreg = b.reg.size();
            int st = ST_OK;
            if (nreg) {
                uint8_t *hbuf = B.host(b.slot == 0 ? Buffers::HOST_IN : Buffers::HOST_IN2, b.hbytes + 64);
                const uint8_t *d_in = hbuf ? upload(B, Buffers::IN, hbuf, b.hbytes, s) : nullptr;
                const uint64_t *d_rec = reinterpret_cast<const uint64_t *>(
                    upload(B, Buffers::REC, reinterpret_cast<const uint8_t *>(b.roff.data()), 8 * b.roff.size(), s));
                if (!d_in || !d_rec) st = ST_E_HIP;
                std::vector<uint64_t> lend;
                uint64_t j0 = 0;
                while (!st && j0 < nreg) {
                    int stop_at = 0;
                    uint64_t cont = 0;
                    lend.clear();
                    const uint64_t base = L.size();
                    auto lsink = [&](const uint8_t *p, uint64_t k) { L.insert(L.end(), p, p + k); return true; };
                    st = decode_records(d_in, b.hbytes, S, d_rec + j0, nullptr, nreg - j0, B, s, lsink, 1ull << 30,
                                        &stop_at, &cont, &lend);
                    if (st) break;
                    uint64_t got = lend.size();
                    if (stop_at == 2) { got--; L.resize(base + (got ? lend[got - 1] : 0)); }   // its line read past the record
                    for (uint64_t k = 0; k < got; k++) {
                        const uint64_t i = b.reg[j0 + k];
                        lo[i] = base + (k ? lend[k - 1] : 0);
                        le[i] = base + lend[k];
                        pend[i] = b.recs[i].ls + 16 + (b.roff[j0 + k + 1] - b.roff[j0 + k]);
                    }
                    if (stop_at == 0) break;
                    j0 += got + 1;   // the stopping record: window path below
                }
            }
            free_slots.put(b.slot);   // its bytes are on the device (decode_records synchronised)
            tr.dec += Trace::now() - t0;
            if (st) { status = st; free_lines.put(lb); more = false; break; }
            // verdicts in order; accepted lines that lie back to back in L form one span
            t0 = Trace::now();
            WriteJob job;
            job.buf = lb;
            bool done = false;
            for (uint64_t i = 0; i < nr && !done; i++) {
                const SqRec &r = b.recs[i];
                if (r.walk) { status = r.walk; done = true; break; }
                if (lo[i] == ~0ull) {   // window path: its line goes to the end of L
                    std::vector<uint8_t> one;
                    if ((st = sq_line_window(fd, fsize, r.ls + 16, S, B, s, one, &pend[i]))) { status = st; done = true; break; }
                    lo[i] = L.size();
                    L.insert(L.end(), one.begin(), one.end());
                    le[i] = L.size();
                }
                const uint8_t *x = L.data() + lo[i];
                const uint64_t n = le[i] - lo[i];
                // SplitIterator(line, "\t"): CHROM, POS (split_iterator.cpp); strtoul whole (:520-524)
                uint64_t t1 = 0;
                while (t1 < n && x[t1] != '\t') t1++;
                uint64_t t2 = t1 + 1, pos = 0;
                while (t2 < n && x[t2] != '\t') t2++;
                if (t1 >= n || !sq_strtoul_whole(x + t1 + 1, t2 - t1 - 1, &pos)) {   // no second term / bad POS: throws
                    status = ST_E_FORMAT;
                    done = true;
                    break;
                }
                if (!(t1 == q.ref_len && memcmp(x, q.ref, q.ref_len) == 0 && pos <= q.end)) { done = true; break; }
                if (!job.spans.empty() && job.spans.back().second == lo[i]) job.spans.back().second = le[i];
                else job.spans.emplace_back(lo[i], le[i]);
                if (r.dnext == 0 || pos >= q.end) { done = true; break; }
                if (r.sync) { ls = pend[i]; resume = true; }   // the failed lseek leaves the parse end
            }
            tr.eval += Trace::now() - t0;
            jobs.put(std::move(job));
            if (done) { more = false; break; }
            if (b.last) { more = resume; break; }   // a sync record: walk on from its parse end
        }
        finish_walker();
        tr.walk += walk_t;
    }
    jobs.close();
    writer.join();
    tr.total = Trace::now() - t_begin;
    if (status == ST_OK && write_failed) status = ST_E_IO;
    return status;
}

inline int sparse_query(int fd, const SparseQuery &q, Buffers &B, hipStream_t s, const Sink &sink,
                        bool trace = false) {
    struct stat sb;
    if (fstat(fd, &sb) != 0) return ST_E_IO;
    const uint64_t fsize = (uint64_t)sb.st_size;
    // decompress2_metadata_headers_fd (compress.cpp:1108-1211) over a growing prefix
    uint64_t data = 0, S = 0;
    std::vector<uint8_t> hb;
    for (uint64_t hn = 1ull << 16;; hn *= 4) {
        hb.resize(std::min(hn, fsize));
        const int64_t got = sq_pread(fd, hb.data(), hb.size(), 0);
        if (got < 0) return ST_E_IO;
        if (parse_header(hb.data(), (uint64_t)got, &data, &S) == ST_OK) break;
        if ((uint64_t)got >= fsize) return ST_E_FORMAT;
    }
    const int64_t data_start = (int64_t)data + 8;   // main.cpp:263-267
    uint8_t fb[8] = {0};
    if (sq_pread(fd, fb, 8, data) < 8) return ST_E_FORMAT;   // :268-272
    uint64_t first = 0;
    for (int i = 7; i >= 0; i--) first = (first << 8) | fb[i];   // host (little-endian) order
    const bool has_criteria = q.ref_len > 0 || q.has_range;
    if (!has_criteria) return ST_E_FORMAT;   // "sparse query with no filter is not yet implemented"
    std::vector<uint8_t> line;
    if (q.start == q.end) {
        // single variant lookup (:278-333): the line at the slot, unfiltered
        const off_t nw = (off_t)((uint64_t)data_start + sq_slot(q.start));
        if (lseek(fd, nw, SEEK_SET) != nw) return ST_OK;   // perror, return
        uint8_t h[16] = {0};   // (a short read leaves stack bytes there; zero here)
        const int64_t k = sq_pread(fd, h, 16, (uint64_t)nw);
        if (k < 0) return ST_E_IO;
        if (k == 0) return ST_E_FORMAT;   // "Reached end of file unexpectedly"
        if (sq_be64(h) == 0 && nw != (off_t)(first + (uint64_t)data_start)) return ST_OK;
        uint64_t end = 0;
        const int st = sq_line_window(fd, fsize, (uint64_t)nw + (uint64_t)k, S, B, s, line, &end);
        if (st) return st;
        return sink(line.data(), line.size()) ? ST_OK : ST_E_IO;
    }
    // range (:335-421): the slot of start, SEEK_DATA, the next slot boundary,
    // then slots whose dist_to_prev is 0 are holes (unless the first line's)
    const off_t init = lseek(fd, (off_t)((uint64_t)data_start + sq_slot(q.start)), SEEK_SET);
    const off_t sd = lseek(fd, init, SEEK_DATA);
    if (sd < init) return ST_E_FORMAT;
    if (init != sd && (sd - data_start) % SQ_STRIDE != 0) {
        const off_t nx = SQ_STRIDE - ((sd - data_start) % SQ_STRIDE);
        const off_t cur = lseek(fd, 0, SEEK_CUR);
        if (lseek(fd, nx, SEEK_CUR) != nx + cur) return ST_OK;   // perror, return
    }
    for (;;) {
        uint8_t h[16] = {0};
        const ssize_t k = read(fd, h, 16);
        if (k < 16) return ST_E_FORMAT;
        if (sq_be64(h) == 0 && init != (off_t)(first + (uint64_t)data_start)) {
            lseek(fd, SQ_STRIDE - 16, SEEK_CUR);
        } else {
            lseek(fd, -16, SEEK_CUR);
            break;
        }
    }
    return sq_traverse(fd, fsize, (uint64_t)lseek(fd, 0, SEEK_CUR), S, q, B, s, sink, trace);
}

}  // namespace vcfc_dec
