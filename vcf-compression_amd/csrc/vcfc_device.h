// vcfc_device.h -- device-side launch interface shared by the C-ABI
// (vcfc_api.cpp) and the kernels (vcfc_encode.hip).  Plain pointers only.
#pragma once
// The kernels' diagnostic switches make libvcfc.so write WRONG .vcfc bytes
// (they remove steps to price them: profiles/r04/ab/*bisect*).  They exist for
// the A/B builds under build_ab/ only, which must also define
// VCFC_DIAG_BUILD; a product build with any of them is refused here (and by
// the Makefile, tests/test_capi.py::test_diag_switches_refused).
#if (defined(VCFC_DIAG_NOSTORE) || defined(VCFC_DIAG_NOSTEP) || defined(VCFC_DIAG_CLEAN_SKIP) || \
     defined(VCFC_VAR_SIZE_ONLY) || defined(VCFC_DIAG_DEC_NOSCAN) || defined(VCFC_DIAG_NOESCEMIT) || \
     defined(VCFC_DIAG_NODIRECT) || defined(VCFC_DIAG_HOP_TWICE)) && \
    !defined(VCFC_DIAG_BUILD)
#error "VCFC_DIAG_* / VCFC_VAR_SIZE_ONLY produce wrong output: diagnostic builds only (define VCFC_DIAG_BUILD)"
#endif
#include <stddef.h>
// deferred records on (1) or off (0) by default (A/B builds set 0)
#ifndef VCFC_DEFER_DEFAULT
#define VCFC_DEFER_DEFAULT 1
#endif
#include <stdint.h>
#include <hip/hip_runtime.h>

// status codes (identical to include/vcfc.h)
#define VCFCD_OK 0
#define VCFCD_E_LT8COLS 1
#define VCFCD_E_8COLS 2
#define VCFCD_E_NOSPACE 4
// a row holding a '\n' byte, seen only when VcfcEncodeArgs::nl_check is set:
// the hop line index (vcfc_line_index with S_hint) mispredicted a line end
#define VCFCD_E_NEWLINE 9
// a deferred record came out another size than it was sized (cannot happen;
// reported as VCFC_E_HIP, a device failure)
#define VCFCD_E_INTERNAL 6
// a line longer than VCFCD_MAX_LINE (include/vcfc.h VCFC_E_TOOLONG): records
// stay below 2^30 bytes, the LEN header's range, so that every rec_size flag
// below (VCFCD_RETRY_GT, VCFCD_DEFER: the top two bits) is free of sizes
#define VCFCD_E_TOOLONG 10
#define VCFCD_MAX_LINE ((1u << 29) - 64u)

// error word: min over failing rows of (row << 8 | code); ~0 = no error
#define VCFCD_NO_ERROR (~0ull)
// rec_size value of a row the fast kernel leaves to k_encode_var
#define VCFCD_RETRY 0xFFFFFFFFu
// ... or, when k_encode_fast parsed a clean prefix inside the line's first
// 1 KiB and only the genotype tokens were of another shape, VCFCD_RETRY_GT |
// the first sample's offset (< VCFCD_GT0_NONE): k_encode_var skips the parse
#define VCFCD_RETRY_GT 0xC0000000u
#define VCFCD_GT0_NONE 0x3FFFFFFFu
// ... with this bit when the row starts with escapes -- its first token is 5
// bytes or longer (GT:DP:GQ and the like), or every token of its first 2 KiB
// genotype chunk is a 3-byte escape (unphased "0/1", "./."): with deferred
// records k_encode_var predicts its record without reading it (the offset
// itself is < 1 KiB)
#define VCFCD_GT0_LONG 0x20000000u
// rec_size flag of a deferred row: k_encode_var only sized it (every chunk an
// escape chunk), k_encode_defer writes its record straight to out after the
// size scan (the size is the low 31 bits)
#define VCFCD_DEFER 0x80000000u

// Alignment: buf, the lines in it and out may start at any byte.  The
// kernels address them with 16-byte loads and stores at the base's own
// alignment (k_nl_scan reads a chunk from d_in + pos, k_nl_hop a line's
// windows from any byte of it, k_compact_out stores
// 16-B blocks at out + 16k, out = d_out + header bytes in compress_device);
// gfx950 global and buffer memory instructions take unaligned addresses (ROCm
// runs the GPU with SH_MEM_CONFIG's unaligned mode), an unaligned base only
// costs the split accesses.  tests/test_gpu_ingest.py and test_kernel_emu.py
// run unaligned bases and chunk starts (all 16 alignments of the buffer).
struct VcfcEncodeArgs {
    // input: concatenated VCF data lines (device memory)
    const uint8_t *buf;
    const uint64_t *line_off;  // byte offset of line i in buf
    const uint32_t *line_len;  // length of line i, without '\n'
    uint64_t n;                // rows
    uint64_t line_bytes_hint;  // sum of the line lengths (<= the workspace's total_line_bytes): picks the compaction shape
    // output
    uint8_t *out;              // records, concatenated in row order
    uint64_t out_cap;
    uint64_t *rec_off;         // n + 1 exclusive offsets; rec_off[n] = total
    // workspace (see vcfc_encode_workspace_layout)
    uint64_t *slot_off;        // n + 1
    uint32_t *rec_size;        // n
    uint64_t *partials;        // scan partials
    uint64_t *err;             // 1 word
    uint32_t *retry_count;     // rows that took the general path (emulator builds only, diag hooks)
    uint32_t *defer_count;     // deferred rows (VCFCD_DEFER), zeroed per encode with lb
    uint32_t *defer_list;      // their row indices (any order), n entries
    // predicted deferred records (k_encode_var sizes an all-escape row from
    // its first chunk and the token count two earlier rows agreed on;
    // k_encode_defer's first pass checks every record against its size):
    uint32_t *mispredict;      // nonzero: some record's size was wrong -- the size scan, compaction and
                               // deferred writes run again on the exact sizes (gated launches)
    uint32_t *defer_fallback;  // deferred rows not written straight to out: the general path after all, a '\n', the cap
    uint64_t *nospace;         // the first size scan's out_cap report (row << 8 | VCFCD_E_NOSPACE),
                               // merged into err unless the scan runs again
    uint8_t *lb;               // look-back scan state (tickets, tile flags; zeroed per encode)
    uint32_t *tile_first;      // per 4 KiB output tile: the row holding its first byte (compaction)
    uint8_t *prim;             // per-row primary staging: record bytes [0, prim_bytes) at prim + prim_bytes * row
    uint8_t *slots;            // per-row overflow slots: record bytes [prim_bytes, ...) at slots + slot_off[row]
    uint32_t prim_bytes;       // vcfc_prim_bytes of the workspace layout
    uint64_t slots_cap;
    uint64_t *dbg;             // diagnostic builds only (tools/diag hooks); else null
    // rows from the hop line index: a row holding a '\n' fails with
    // VCFCD_E_NEWLINE (k_encode_var scans the rows k_encode_fast hands back;
    // k_encode_fast accepts none)
    uint32_t nl_check = 0;
    // deferred records (k_encode_var sizes the rows whose first genotype
    // chunk is all escapes and that span more than one chunk, k_encode_defer
    // writes them to out after the size scan): on by
    // default since round 5 -- the choice is made per row by the kernel from
    // the row's own bytes, and a batch without such rows pays one empty
    // launch; vcfc_ctx_set_deferred_records(ctx, 0) turns it off
    uint32_t defer_records = VCFC_DEFER_DEFAULT;
};

// Record staging: the first prim_bytes bytes of every record go to a dense
// per-row array (the compaction then reads most records from consecutive
// kilobytes), the rest (records of rare escape-heavy rows) to a per-row
// overflow slot sized for the worst case.  2 KiB for batches of long lines
// (mean >= 4 KiB: records of 1-2 KiB, e.g. the random_vcf law's ~1.28 KB at
// 2504 samples, stay in one region; k_compact -14 % on law 0 and -9 % on
// law 1 in an A/B, 4 KiB slower again, profiles/r03/ab/ab_prim*.txt), else
// 1 KiB (the region costs prim_bytes per row whatever the line length).
// A multiple of the 1 KiB flush burst, so no burst straddles the regions.
__host__ __device__ inline uint32_t vcfc_prim_bytes(uint64_t n, uint64_t total_line_bytes) {
    return n && total_line_bytes / n >= 4096 ? 2048u : 1024u;
}

struct VcfcWorkspaceLayout {
    uint64_t slot_off, rec_size, partials, err, lb, lb_bytes, retry_count, defer_count, mispredict, defer_fallback,
        nospace, defer_list, tile_first, prim, slots, dbg, total;
    uint32_t prim_bytes;
};

// Bytes of per-row staging for a line of `len` bytes: covers the worst-case
// record (8 + len + (len+1)/2 + 2) plus the 16-byte flush granule.
__host__ __device__ inline uint64_t vcfc_slot_bytes(uint32_t len) {
    return ((uint64_t)len + (len >> 1) + 48 + 15) & ~15ull;
}

// Upper bound of the records of n rows whose line bytes sum to total
// (include/vcfc.h vcfc_encode_bound).
__host__ __device__ inline uint64_t vcfc_record_bound(uint64_t n, uint64_t total) {
    return total + total / 2 + 16 * n + 16;
}

// Workspace layout for n rows whose line lengths sum to <= total_line_bytes.
VcfcWorkspaceLayout vcfc_encode_workspace_layout(uint64_t n, uint64_t total_line_bytes);

// Point a's workspace arrays into ws (err is the caller's).
inline void vcfc_encode_args_workspace(VcfcEncodeArgs &a, uint8_t *ws, const VcfcWorkspaceLayout &L) {
    a.slot_off = reinterpret_cast<uint64_t *>(ws + L.slot_off);
    a.rec_size = reinterpret_cast<uint32_t *>(ws + L.rec_size);
    a.partials = reinterpret_cast<uint64_t *>(ws + L.partials);
    a.retry_count = reinterpret_cast<uint32_t *>(ws + L.retry_count);
    a.defer_count = reinterpret_cast<uint32_t *>(ws + L.defer_count);
    a.defer_list = reinterpret_cast<uint32_t *>(ws + L.defer_list);
    a.mispredict = reinterpret_cast<uint32_t *>(ws + L.mispredict);
    a.defer_fallback = reinterpret_cast<uint32_t *>(ws + L.defer_fallback);
    a.nospace = reinterpret_cast<uint64_t *>(ws + L.nospace);
    a.lb = ws + L.lb;
    a.tile_first = reinterpret_cast<uint32_t *>(ws + L.tile_first);
    a.prim = ws + L.prim;
    a.prim_bytes = L.prim_bytes;
    a.slots = ws + L.slots;
    a.slots_cap = L.dbg - L.slots;
    a.dbg = L.dbg < L.total ? reinterpret_cast<uint64_t *>(ws + L.dbg) : nullptr;
}

// Rows the last encode on this workspace deferred (the device word behind
// VcfcEncodeArgs::defer_count; read by the caller after the stream is done).
inline uint64_t vcfc_defer_count_offset(const VcfcWorkspaceLayout &L) { return L.defer_count; }
// ... of which this many were written by the general path after all (a
// predicted all-escape row whose later chunks had another shape)
inline uint64_t vcfc_defer_fallback_offset(const VcfcWorkspaceLayout &L) { return L.defer_fallback; }

// Enqueue the whole encode on `stream` (no host synchronisation, capturable).
// If `ev` is non-null, ev[0..5] are recorded before the slot scan, after it,
// after k_encode (fast + variable-token kernels), after the size scan, after
// k_compact and after k_encode_defer.
hipError_t vcfc_encode_device(const VcfcEncodeArgs &a, hipStream_t stream, hipEvent_t *ev = nullptr);

// ---------------------------------------------------------------------------
// Decoder (vcfc_decode.hip).  Records of one batch, located by LEN hops.
struct VcfcDecodeArgs {
    const uint8_t *in;          // data section bytes (device)
    uint64_t n_bytes;           // bytes available from `in` (the byte-serial parse may read past a record)
    const uint64_t *rec_start;  // n + 1 record offsets into `in` (rec_start[n] = end of the hopped range)
    const uint8_t *select;      // nullptr, or per record: 0 = skip it (no line; the range query's non-matches)
    uint64_t n;                 // records
    uint64_t S;                 // samples declared by the header line
    uint8_t *out;               // decoded lines, concatenated
    uint64_t out_cap;
    uint64_t *line_off;         // n + 1 exclusive offsets of the lines in `out`
    // workspace (vcfc_decode_workspace_layout)
    uint32_t *st;               // per-record plan status
    uint32_t *line_size;        // per-record line bytes
    uint64_t *end;              // byte-serial parse end (queued records)
    uint32_t *seq_list;         // records queued for the byte-serial path
    uint32_t *seq_count;
    uint64_t *err;              // min over records of (i << 8 | code): 2 = parse ends off the hop, 3 = reference error,
                                // 4 = light plan was wrong (rerun exactly), 0xFF = out_cap short
    uint64_t *partials;         // scan partials
};

struct VcfcDecodeLayout {
    uint64_t st, line_size, end, seq_list, seq_count, err, partials, total;
};

VcfcDecodeLayout vcfc_decode_workspace_layout(uint64_t n);
// plan: statuses, sizes, line offsets (no host synchronisation).  exact =
// false scans only headers and REQ and assumes the sample sections are
// simple; k_dec_write then reports (i << 8 | 4) in err for a record where
// that was wrong, and the batch must be planned again with exact = true.
hipError_t vcfc_decode_plan(const VcfcDecodeArgs &a, bool exact, hipStream_t s);
// write lines [first, last) at a.out + line_off[i] (their plan status must not be an error)
hipError_t vcfc_decode_write(const VcfcDecodeArgs &a, uint64_t first, uint64_t last, hipStream_t s);
// one-lane byte-serial decode of in[p, n), at most max_lines lines: out ==
// nullptr counts; st[0..3] = {0 max_lines reached | 1 clean end | 2 reference
// error, bytes, lines, parse end}
hipError_t vcfc_decode_stream(const uint8_t *in, uint64_t n, uint64_t p, uint64_t S, uint64_t max_lines,
                              uint8_t *out, uint64_t *st, hipStream_t s);
// per-record 64-bit digests of records[rec_off[i], rec_off[i + 1]) (vcfc_check.hip)
hipError_t vcfc_record_hash(const uint8_t *recs, const uint64_t *rec_off, uint64_t n, uint64_t *out, hipStream_t s);
// exclusive u32 -> u64 scan with out[n] = total (shared with the encoder)
hipError_t vcfc_scan_u32(const uint32_t *in, uint64_t n, uint64_t *partials, uint64_t *out, hipStream_t s);
// The same over line kinds (bit 0: data line, bit 1: '#' line): out[i] =
// data lines before i | '#' lines before i << 32 (line index phase 2).
hipError_t vcfc_scan_kinds(const uint32_t *in, uint64_t n, uint64_t *partials, uint64_t *out, hipStream_t s);

// ---------------------------------------------------------------------------
// Range query (vcfc_decode.hip; reference query_compressed_file,
// src/main.cpp:3777-3929).  `ref` is device memory.
struct VcfcQuery {
    const uint8_t *ref;   // reference name; ref_len == 0 matches every name
    uint32_t ref_len;
    uint32_t has_range;   // 0: name only
    uint64_t start, end;  // inclusive position range
};
// one lane per record [rec_start[i], rec_start[i + 1]): flag[i] = 1 if the
// record matches; err = min over records of (i << 8 | code), code 2 = its
// POS does not parse (the reference throws), 3 = its CHROM or POS field runs
// past the record (the reference's walk leaves the LEN hops: continue with
// vcfc_query_stream from record i)
hipError_t vcfc_query_match(const uint8_t *in, const uint64_t *rec_start, uint64_t n, const VcfcQuery &q,
                            uint8_t *flag, uint64_t *err, hipStream_t s);
// one-lane byte-serial query of in[p, n) (st as vcfc_decode_stream)
hipError_t vcfc_query_stream(const uint8_t *in, uint64_t n, uint64_t p, uint64_t S, const VcfcQuery &q, uint8_t *out,
                             uint64_t *st, hipStream_t s);

// ---------------------------------------------------------------------------
// Line index of an input chunk (vcfc_ingest.hip; reference compress()'s
// getline loop, src/compress.cpp:218-238).
struct VcfcLineIndex {
    uint64_t *line_off;     // data line j: chunk offset, length, 0-based line number in the chunk
    uint32_t *line_len;
    uint32_t *line_no;
    uint64_t *pass_off;     // '#' line q: chunk offset, length, line number, data lines before it
    uint32_t *pass_len;
    uint32_t *pass_no;
    uint64_t *pass_before;
    uint64_t *counts;       // {lines, data lines, pass lines, a line of >= 4 GiB}
};
struct VcfcLineIndexLayout {
    uint64_t seg_cnt, seg_base, slot, wstart, partials1, total1;     // phase 1 workspace
    uint64_t nl, kind, rank, partials2, total2;   // phase 2 workspace
};
VcfcLineIndexLayout vcfc_line_index_layout(uint64_t chunk_bytes, uint64_t n_lines);
// phase 1: '\n' count of buf[0, n) (last byte '\n'); counts[0] = lines.
// S_hint (the header's sample count, 0: none) selects the hop index
// (k_nl_hop: data line ends predicted from S and checked) over the full
// '\n' scan; its result must be confirmed by the encoder (VcfcEncodeArgs::nl_check).
// hop_walkers: walkers of the hop index (0: HOP_WALKERS; the tests use a few,
// so each walks as many lines as at config size).  hop_learn: the walkers
// learn the genotype-region lengths of lines that are not 3-byte tokens
// (TRY / LEARN, k_nl_hop<true>).  len_hint (!hop_learn; 0: none): a data
// line's length with its '\n' (the file's first): every walker but the
// first guesses its first lines from it (GUESS) instead of reading the
// first line's prefix.
// Learned candidates handed to every TRY / LEARN walker at its start (the
// host's: data lines of the file's first window whose genotype region is not
// 4 S - 1 bytes): region length g[k] (0: none) and, for each of the 16 lanes
// of a walker, the TAB mask of its 16 bytes of the 256 ending at the '\n'.
struct VcfcHopCands {
    uint32_t g[3];
    uint16_t sig[3][16];
};
hipError_t vcfc_line_index(const uint8_t *buf, uint64_t n, uint8_t *ws, const VcfcLineIndexLayout &L,
                           const VcfcLineIndex &x, hipStream_t s, uint32_t S_hint = 0, uint64_t hop_walkers = 0,
                           bool hop_learn = true, uint32_t len_hint = 0, const VcfcHopCands *cands = nullptr);
// phase 2 (n_lines = counts[0]): '\n' positions, data / pass line arrays; counts[1], counts[2]
hipError_t vcfc_line_index_place(const uint8_t *buf, uint64_t n, uint64_t n_lines, const uint8_t *ws1, uint8_t *ws2,
                                 const VcfcLineIndexLayout &L, const VcfcLineIndex &x, hipStream_t s);
// counts[0..3] and the first pk '#' line entries into out (32 + 24 pk bytes)
hipError_t vcfc_index_summary(const VcfcLineIndex &x, uint64_t pk, uint8_t *out, hipStream_t s);
