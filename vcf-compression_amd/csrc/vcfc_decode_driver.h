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
#include <cstdint>
#include <functional>
#include <vector>

#include "vcfc_device.h"

namespace vcfc_dec {

constexpr int ST_OK = 0, ST_E_HIP = 6, ST_E_IO = 7, ST_E_FORMAT = 8;   // = include/vcfc.h codes

// Device buffers, owned by the caller (one slot each; contents not kept).
struct Buffers {
    virtual ~Buffers() {}
    enum { IN = 0, REC, WS, OUT, LINE_OFF, SMALL, FLAG, QREF, N_SLOTS };
    virtual void *get(int slot, uint64_t bytes) = 0;   // nullptr on failure
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
// all records decoded.
inline int decode_records(const uint8_t *d_in, uint64_t n, uint64_t S, const uint64_t *d_rec, const uint8_t *d_select,
                          uint64_t nrec, Buffers &B, hipStream_t s, const Sink &sink, uint64_t out_batch, int *stop,
                          uint64_t *cont) {
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
    std::vector<uint8_t> host;
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
        host.resize(bytes);
        if (hipMemcpyAsync(host.data(), d_out, bytes, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            return ST_E_HIP;
        if (!sink(host.data(), bytes)) return ST_E_IO;
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
    return stream_tail(B, s, sink, [&](uint8_t *out, uint64_t *dst) { return vcfc_decode_stream(d_in, n, p_stream, S, out, dst, s); });
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

}  // namespace vcfc_dec
