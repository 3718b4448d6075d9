// vcfc_decode.hip -- gfx950 kernels for the .vcfc decoder.
//
// Replaces decompress2_data_line (reference src/compress.cpp:741-986) for a
// batch of records resident in HBM.  The reference parses the data section
// byte by byte and never reads a record's LEN header; here the host finds
// record starts by hopping LEN headers, and every record's parse is checked
// to end exactly where the next hop lands.  Where it does not (a record with
// fewer or more samples than the header declares), the rest of the input is
// decoded by k_dec_stream, one lane walking the bytes exactly as the
// reference does.
//
//   k_dec_plan   one wave per record: is the record "simple"?  Then its line
//                is REQ' + 4 * S bytes.  Others are queued for k_dec_seq.
//   k_dec_seq    one lane per queued record: byte-serial parse (size, end,
//                reference error).
//   scan         line offsets (the encoder's exclusive scan).
//   k_dec_write  one wave per record: simple records by an item-driven fill
//                (each run byte writes its tokens as repeated 4-byte words);
//                queued records by the byte-serial writer on lane 0.
//   k_dec_stream one lane: byte-serial decode of a byte range.
//
// A record is simple when: header bits and REQ are sane; REQ holds exactly 9
// TABs; S > 0; the sample section is a sequence of items -- run bytes with a
// non-zero count (0|0: b < 0x80, count b; 0|1 1|0 1|1: 0x80..0xDF, count
// b & 0x1F) and escapes 0xE1 + 3 ASCII bytes (no TAB/LF) + TAB (or the final
// LF) -- whose token counts add up to exactly S; the record's last byte is LF.
// Then every sample token is 3 bytes and the line is REQ' (the C string of
// the REQ bytes: `linebuf.append(buf)` stops at a NUL, compress.cpp:798),
// then S four-byte words "a|b\t" with the last TAB replaced by LF.
#include <hip/hip_runtime.h>
#include <vcfc_wave.h>   // angle brackets: tests/simt_emu shadows it
#include "vcfc_device.h"

namespace {

constexpr int DEC_WAVES = 4;   // records per 256-thread block

// per-record status after planning
constexpr uint32_t DS_SIMPLE = 0;   // line = REQ' + 4S bytes, item fill
constexpr uint32_t DS_SEQ = 1;      // byte-serial path, consistent end
constexpr uint32_t DS_INCONS = 2;   // byte-serial parse ends off the LEN hop
constexpr uint32_t DS_ERR = 3;      // the reference throws at this record

// result of dec_line_seq
constexpr int DL_OK = 0, DL_END = 1, DL_ERR = 2;

__device__ __forceinline__ uint32_t be30(const uint8_t *h) {
    return ((uint32_t)(h[0] & 0x3Fu) << 24) | ((uint32_t)h[1] << 16) | ((uint32_t)h[2] << 8) | h[3];
}

// One data line, byte-serial, exactly as decompress2_data_line
// (compress.cpp:741-986): from the 8 header bytes at in[p] through the
// closing LF.  Writes the line to `out` when non-null.  DL_END: fewer than 8
// bytes left (read_compressed_line_length_headers returns short, :768-774).
__device__ int dec_line_seq(const uint8_t *in, uint64_t n, uint64_t p, uint64_t S, uint8_t *out,
                            uint64_t *size, uint64_t *end) {
    if (n - p < 8) return DL_END;
    const uint8_t *h = in + p;
    if ((h[0] >> 6) != 3u || (h[4] >> 6) != 3u) return DL_ERR;     // utils.hpp:198-206
    const uint32_t req = be30(h + 4);
    uint64_t ip = p + 8, o = 0;
    if (req == 0 || n - ip < req) return DL_ERR;                   // :790-797
    uint64_t tabs = 0;
    bool nul = false;
    for (uint32_t i = 0; i < req; i++) {
        const uint8_t b = in[ip + i];
        tabs += b == '\t';
        nul = nul || b == 0;
        if (!nul) {
            if (out) out[o] = b;
            o++;
        }
    }
    ip += req;
    if (tabs != 9 && !(tabs == 8 && S == 0)) return DL_ERR;        // :818-828
    uint64_t got = 0;
    while (got < S) {                                               // :832-954
        if (ip >= n) return DL_ERR;
        const uint8_t b = in[ip++];
        if ((b & 0x80u) == 0) {
            const uint32_t cnt = b & 0x7Fu;
            for (uint32_t k = 0; k < cnt; k++) {
                if (out) { out[o] = '0'; out[o + 1] = '|'; out[o + 2] = '0'; out[o + 3] = '\t'; }
                o += 4;
            }
            got += cnt;
            if (got >= S && o > 0) o--;                             // pop the last tab
        } else if ((b & 0xE0u) == 0xE0u) {
            const uint32_t uc = b & 0x1Fu;
            uint32_t u = 0;
            while (u < uc) {
                if (ip >= n) return DL_ERR;
                const uint8_t x = in[ip++];
                if (x == '\n') {
                    u++; got++;
                    if (u != uc) return DL_ERR;
                    ip--;                                           // re-read as the line end
                } else if (x == '\t') {
                    u++; got++;
                    if (got < S) { if (out) out[o] = '\t'; o++; }
                } else {
                    if (out) out[o] = x;
                    o++;
                }
            }
        } else {
            const uint32_t m = b & 0xE0u;
            const uint8_t a = m == 0xA0u ? '0' : '1';               // 0|1 -> 0xA0, 1|0 -> 0xC0, 1|1 -> 0x80
            const uint8_t c = m == 0xC0u ? '0' : '1';
            uint32_t cnt = b & 0x1Fu;
            while (cnt--) {
                if (out) { out[o] = a; out[o + 1] = '|'; out[o + 2] = c; }
                o += 3;
                got++;
                if (got < S) { if (out) out[o] = '\t'; o++; }
            }
        }
    }
    if (ip >= n) return DL_ERR;                                     // :958-966
    if (in[ip++] != '\n') return DL_ERR;
    if (out) out[o] = '\n';
    o++;
    *size = o;
    *end = ip;
    return DL_OK;
}

// Wave-parallel scan of a record's sample items (see the header comment).
// Visits each item start with (lane-local) byte b, position k, tokens before
// it (gb) and its count; returns false if the record is not simple.
struct ItemScan {
    const uint8_t *in;
    uint64_t s0, s1;   // sample section [s0, s1); in[s1] is the record's LF
};

template <class F>
__device__ __forceinline__ bool scan_items(const ItemScan &sc, uint64_t S, uint64_t *got_out, F &&visit) {
    const uint32_t l = vw::lane_id();
    uint64_t got = 0, pcarry = 0, tcarry = 0;
    bool bad = false;
    for (uint64_t b0 = sc.s0; b0 < sc.s1; b0 += 64) {
        const uint64_t k = b0 + l;
        const bool valid = k < sc.s1;
        const uint32_t b = valid ? sc.in[k] : 0u;
        const uint64_t E = vw::ballot(valid && b == 0xE1u);
        // payload: the 3 bytes after an escape flag; terminator: the 4th
        const uint64_t P = (E << 1) | (E << 2) | (E << 3) | pcarry;
        const uint64_t TM = (E << 4) | tcarry;
        const uint64_t e = E >> 60;
        pcarry = (e >> 1) | (e >> 2) | (e >> 3);
        tcarry = e;
        const bool is_p = (P >> l) & 1ull, is_t = (TM >> l) & 1ull;
        bool lb = false;
        if (valid) {
            if (is_p) lb = b >= 0x80u || b == '\t' || b == '\n';
            else if (is_t) lb = b != '\t';
            else lb = (b & 0xE0u) == 0xE0u && (b != 0xE1u || k + 4 > sc.s1);   // escape needs 3 bytes + TAB/final LF
        }
        const bool start = valid && !is_p && !is_t;
        const uint32_t cnt = !start ? 0u : b == 0xE1u ? 1u : b < 0x80u ? b : (b & 0x1Fu);
        lb = lb || (start && cnt == 0);
        bad = bad || vw::ballot(lb) != 0;
        const uint32_t inc = vw::scan_add(cnt);
        const uint64_t gb = got + (inc - cnt);
        if (!bad && start) visit(b, k, gb, cnt);
        got += vw::readlane(inc, 63);
    }
    *got_out = got;
    return !bad && got == S;
}

// REQ bytes: TAB count and the C-string length (first NUL).
__device__ __forceinline__ void scan_req(const uint8_t *r, uint32_t req, uint32_t *tabs, uint32_t *slen) {
    const uint32_t l = vw::lane_id();
    uint32_t t = 0, z = req;
    for (uint32_t b0 = 0; b0 < req; b0 += 64) {
        const uint32_t k = b0 + l;
        const uint32_t b = k < req ? r[k] : 0xFFu;
        t += (uint32_t)vw::popc64(vw::ballot(b == '\t'));
        const uint64_t zm = vw::ballot(b == 0);
        if (zm && z == req) z = b0 + (uint32_t)__builtin_ctzll(zm);
    }
    *tabs = t;
    *slen = z;
}

__global__ __launch_bounds__(256) void k_dec_plan(VcfcDecodeArgs a) {
    const uint32_t wave = vw::readfirst(threadIdx.x >> 6);
    const uint64_t i = (uint64_t)blockIdx.x * DEC_WAVES + wave;
    if (i >= a.n) return;
    const uint64_t rs = a.rec_start[i], re = a.rec_start[i + 1];
    bool simple = false;
    uint64_t size = 0;
    if (re - rs >= 10 && a.S > 0) {
        const uint8_t *h = a.in + rs;
        const uint32_t req = be30(h + 4);
        if ((h[0] >> 6) == 3u && (h[4] >> 6) == 3u && req > 0 && 9 + (uint64_t)req < re - rs &&
            a.in[re - 1] == '\n') {
            uint32_t tabs, slen;
            scan_req(h + 8, req, &tabs, &slen);
            if (tabs == 9) {
                uint64_t got;
                ItemScan sc{a.in, rs + 8 + req, re - 1};
                simple = scan_items(sc, a.S, &got, [](uint32_t, uint64_t, uint64_t, uint32_t) {});
                size = slen + 4 * a.S;
            }
        }
    }
    if (vw::lane_id() == 0) {
        a.st[i] = simple ? DS_SIMPLE : DS_SEQ;
        a.line_size[i] = simple ? (uint32_t)size : 0u;
        if (!simple) {
            const uint32_t q = atomicAdd(a.seq_count, 1u);
            a.seq_list[q] = (uint32_t)i;
        }
    }
}

// Queued records, one lane each (grid-stride).
__global__ __launch_bounds__(256) void k_dec_seq(VcfcDecodeArgs a) {
    const uint32_t cnt = *a.seq_count;
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < cnt; q += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = a.seq_list[q];
        const uint64_t rs = a.rec_start[i], re = a.rec_start[i + 1];
        uint64_t size = 0, end = 0;
        const int r = dec_line_seq(a.in, a.n_bytes, rs, a.S, nullptr, &size, &end);
        uint32_t st;
        if (r != DL_OK || size > 0xFFFFFFFFull) st = DS_ERR;
        else st = end == re ? DS_SEQ : DS_INCONS;
        a.st[i] = st;
        a.line_size[i] = st == DS_ERR ? 0u : (uint32_t)size;
        a.end[i] = end;
        if (st >= DS_INCONS) atomicMin((unsigned long long *)a.err, (unsigned long long)((i << 8) | st));
    }
}

__global__ __launch_bounds__(256) void k_dec_write(VcfcDecodeArgs a, uint64_t first, uint64_t last) {
    const uint32_t wave = vw::readfirst(threadIdx.x >> 6);
    const uint64_t i = first + (uint64_t)blockIdx.x * DEC_WAVES + wave;
    if (i >= last) return;
    const uint32_t l = vw::lane_id();
    const uint64_t rs = a.rec_start[i];
    const uint64_t L0 = a.line_off[i];
    if (a.line_off[i + 1] > a.out_cap) {
        if (l == 0) atomicMin((unsigned long long *)a.err, (unsigned long long)((i << 8) | 0xFFu));
        return;
    }
    uint8_t *line = a.out + L0;
    if (a.st[i] == DS_ERR) return;   // no line (size 0); the reference throws here
    if (a.st[i] != DS_SIMPLE) {
        if (l == 0) {
            uint64_t size, end;
            (void)dec_line_seq(a.in, a.n_bytes, rs, a.S, line, &size, &end);
        }
        return;
    }
    const uint8_t *h = a.in + rs;
    const uint32_t req = be30(h + 4);
    const uint64_t re = a.rec_start[i + 1];
    const uint32_t slen = (uint32_t)(a.line_off[i + 1] - L0 - 4 * a.S);   // REQ' = line - 4S
    for (uint32_t k = l; k < slen; k += 64) line[k] = h[8 + k];
    uint8_t *tok = line + slen;
    const uint64_t S = a.S;
    uint64_t got;
    ItemScan sc{a.in, rs + 8 + req, re - 1};
    scan_items(sc, S, &got, [&](uint32_t b, uint64_t k, uint64_t gb, uint32_t cnt) {
        // the item's token as a little-endian word "a|b\t"
        uint32_t w;
        if (b == 0xE1u) {
            w = (uint32_t)a.in[k + 1] | ((uint32_t)a.in[k + 2] << 8) | ((uint32_t)a.in[k + 3] << 16);
        } else if (b < 0x80u) {
            w = 0x307C30u;
        } else {
            const uint32_t m = b & 0xE0u;
            w = (m == 0xA0u ? 0x30u : 0x31u) | 0x7C00u | ((m == 0xC0u ? 0x30u : 0x31u) << 16);
        }
        w |= 0x09000000u;
        uint8_t *p = tok + 4 * gb;
        uint32_t j = 0;
        for (; j + 4 <= cnt; j += 4) vw::gstore16(p, 4ull * j, make_uint4(w, w, w, w));
        if (cnt & 2u) { *reinterpret_cast<uint2 *>(p + 4ull * j) = make_uint2(w, w); j += 2; }
        if (cnt & 1u) *reinterpret_cast<uint32_t *>(p + 4ull * j) = w;
        if (gb + cnt == S) tok[4 * S - 1] = '\n';   // same lane, after its words
    });
}

// Byte-serial decode of [p, n): mode 0 counts (lines, bytes, end state),
// mode 1 writes.  One lane.  st[0] = DL_END (clean end) or DL_ERR; st[1] =
// bytes; st[2] = lines.
__global__ void k_dec_stream(const uint8_t *in, uint64_t n, uint64_t p, uint64_t S, uint8_t *out,
                             uint64_t *st) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint64_t o = 0, lines = 0;
    int r;
    for (;;) {
        uint64_t size = 0, end = 0;
        r = dec_line_seq(in, n, p, S, out ? out + o : nullptr, &size, &end);
        if (r != DL_OK) break;
        o += size;
        p = end;
        lines++;
    }
    st[0] = (uint64_t)r;
    st[1] = o;
    st[2] = lines;
}

}  // namespace

VcfcDecodeLayout vcfc_decode_workspace_layout(uint64_t n) {
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    VcfcDecodeLayout L;
    uint64_t o = 0;
    L.st = o; o = al(o + 4 * (n + 1));
    L.line_size = o; o = al(o + 4 * (n + 1));
    L.end = o; o = al(o + 8 * (n + 1));
    L.seq_list = o; o = al(o + 4 * (n + 1));
    L.seq_count = o; o = al(o + 8);
    L.err = o; o = al(o + 8);
    L.partials = o; o = al(o + 8 * ((n + 4095) / 4096 + 1));
    L.total = o;
    return L;
}

hipError_t vcfc_decode_plan(const VcfcDecodeArgs &a, hipStream_t s) {
    hipError_t e = hipMemsetAsync(a.err, 0xFF, 8, s);
    if (e != hipSuccess) return e;
    if ((e = hipMemsetAsync(a.seq_count, 0, 4, s)) != hipSuccess) return e;
    if (a.n == 0) return hipMemsetAsync(a.line_off, 0, 8, s);
    hipLaunchKernelGGL(k_dec_plan, dim3((unsigned)((a.n + DEC_WAVES - 1) / DEC_WAVES)), dim3(64 * DEC_WAVES), 0, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const uint64_t want = (a.n + 255) / 256;
    hipLaunchKernelGGL(k_dec_seq, dim3((unsigned)(want < 1024 ? want : 1024)), dim3(256), 0, s, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return vcfc_scan_u32(a.line_size, a.n, a.partials, a.line_off, s);
}

hipError_t vcfc_decode_write(const VcfcDecodeArgs &a, uint64_t first, uint64_t last, hipStream_t s) {
    if (last <= first) return hipSuccess;
    hipLaunchKernelGGL(k_dec_write, dim3((unsigned)((last - first + DEC_WAVES - 1) / DEC_WAVES)), dim3(64 * DEC_WAVES), 0,
                       s, a, first, last);
    return hipGetLastError();
}

hipError_t vcfc_decode_stream(const uint8_t *in, uint64_t n, uint64_t p, uint64_t S, uint8_t *out, uint64_t *st,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_dec_stream, dim3(1), dim3(64), 0, s, in, n, p, S, out, st);
    return hipGetLastError();
}
