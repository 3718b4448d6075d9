/*
 * vcfc.h -- C ABI of the MI355X-native `.vcfc` genotype-line codec
 * (libvcfc.so).  Plain pointers and sizes only; no C++ or torch types.
 *
 * Drop-in boundary.  The reference has no FFI: its only boundary for this
 * path is the C++ function
 *     int compress_data_line(const std::string& line,
 *                            const VcfCompressionSchema& schema,
 *                            std::vector<byte_t>& byte_vec, bool add_newline);
 * (reference src/compress.hpp:20-23, defined src/compress.cpp:5-203) whose
 * single caller is compress() (src/compress.cpp:205-257, call at :244).
 * vcfc_compress_data_line() is its one-line replacement; the batch entry
 * points below replace the compress() loop around it.  INTEGRATION.md shows
 * the shim a maintainer adds on the reference side.
 *
 * Output is byte-identical to the reference for every input line: records
 * [LEN][REQ][cols][GT][\n] concatenated in row order (format: reference
 * src/utils.hpp:44-56,140-247, src/compress.cpp:32-199).
 */
#ifndef VCFC_H
#define VCFC_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes -------------------------------------------------------- */
#define VCFC_OK 0
/* VcfValidationError("VCF data line did not contain at least 8 terms"),
 * reference src/compress.cpp:9-11 */
#define VCFC_E_LT8COLS 1
/* exactly 8 terms: the reference's size_t underflow -> std::length_error ->
 * abort (src/compress.cpp:89,107); reported instead of aborting */
#define VCFC_E_8COLS 2
/* VcfValidationError("VCF Header did not have enough columns"),
 * src/compress.cpp:231-234 */
#define VCFC_E_HEADER 3
#define VCFC_E_NOSPACE 4   /* caller buffer too small */
#define VCFC_E_ARG 5       /* bad argument */
#define VCFC_E_HIP 6       /* HIP runtime error / no GPU */
#define VCFC_E_IO 7        /* file open/read/write failed */
#define VCFC_E_FORMAT 8    /* malformed .vcfc input (decoder) */
/* a data line longer than VCFC_MAX_LINE bytes: its record could pass the
 * 30-bit LEN header (LineLengthHeader's 2^30 - 1, reference
 * src/utils.hpp:140-160), which the reference would silently truncate */
#define VCFC_E_TOOLONG 10
#define VCFC_MAX_LINE ((1u << 29) - 64u)

const char *vcfc_version(void);
const char *vcfc_strerror(int status);

/* ---- context ----------------------------------------------------------------
 * One context per GPU (device ordinal); not shared across host threads.
 * Fails with VCFC_E_HIP when no GPU is visible: there is no CPU fallback. */
typedef struct vcfc_ctx vcfc_ctx;
int vcfc_ctx_create(int device, vcfc_ctx **out);
void vcfc_ctx_destroy(vcfc_ctx *ctx);
/* Input chunk of the pipelined file compress (vcfc_compress_file/_buffer):
 * chunk_bytes in [4096, 3 GiB], or 0 for the default (128 MiB).  A line longer
 * than the chunk grows that chunk (doubling) until it fits; no input is read
 * twice.  The reference reads line by line (getline, src/compress.cpp:218);
 * the output does not depend on the chunk size. */
int vcfc_ctx_set_ingest_chunk(vcfc_ctx *ctx, uint64_t chunk_bytes);
/* Line index of vcfc_compress_device: VCFC_LINE_INDEX_HOP (default) guesses
 * each data line's end from the header's sample count and checks it (a wrong
 * guess re-indexes the chunk from every byte, so the output never depends on
 * it); VCFC_LINE_INDEX_SCAN reads every byte.  The reference finds lines with
 * getline (src/compress.cpp:218). */
#define VCFC_LINE_INDEX_HOP 0
#define VCFC_LINE_INDEX_SCAN 1
int vcfc_ctx_set_line_index(vcfc_ctx *ctx, int mode);
/* Stage timings / decisions of the host drivers to stderr (diagnostics; off
 * by default): OR of the flags below. */
#define VCFC_TRACE_INGEST 1u        /* vcfc_compress_file/_buffer/_range: stage totals */
#define VCFC_TRACE_DEVICE 2u        /* vcfc_compress_device: chunks, sample count, re-indexes */
#define VCFC_TRACE_SPARSE_QUERY 4u  /* vcfc_sparse_query*: stage totals */
int vcfc_ctx_set_trace(vcfc_ctx *ctx, unsigned flags);
/* Deferred records (1 = on, the default since round 5; 0 = off) for the
 * context's file and device compress calls (vcfc_encode_rows_device and the
 * one-line / host-batch calls always use them): a row of odd-length tokens
 * whose first genotype chunk is all escapes (GT:DP:GQ and the like, records
 * ~1.1x their lines) and that spans more than one 2 KiB chunk is only sized
 * by the first pass and encoded straight into the output once the record
 * offsets are known, instead of staged and copied.  The choice is made per
 * row by the kernel from the row's bytes; once two rows agree on their token
 * count, a deferred row's size is predicted from its first chunk and checked
 * when it is written (a wrong guess lays the batch out again: three gated
 * launches that return at once otherwise).  Output identical either way
 * (DESIGN.md section 3). */
int vcfc_ctx_set_deferred_records(vcfc_ctx *ctx, int on);

/* ---- one line: replaces compress_data_line (src/compress.hpp:20-23) --------
 * Appends the record for `line` (no trailing '\n'; `len` bytes) to `out`
 * (capacity `out_cap`), writes its size to *out_len.  add_newline as in the
 * reference (compress() always passes true).  Returns VCFC_OK or an error;
 * nothing is written on error. */
int vcfc_compress_data_line(vcfc_ctx *ctx, const char *line, uint64_t len, int add_newline,
                            uint8_t *out, uint64_t out_cap, uint64_t *out_len);

/* ---- batches of lines ------------------------------------------------------
 * Upper bound of the encoded size of rows whose line bytes sum to
 * total_line_bytes (records only). */
uint64_t vcfc_encode_bound(uint64_t n_rows, uint64_t total_line_bytes);

/* Device workspace bytes needed by vcfc_encode_rows_device. */
uint64_t vcfc_encode_workspace_size(uint64_t n_rows, uint64_t total_line_bytes);

/* Device-resident batch encode, asynchronous on `stream` (a hipStream_t; 0 =
 * the default stream).  All pointers are device pointers.
 *   d_buf            data-line bytes
 *   d_line_off/len   line i = d_buf[d_line_off[i] .. + d_line_len[i]) (no '\n')
 *   d_out            records in row order; d_rec_off[0..n] exclusive offsets
 *                    (d_rec_off[n] = total bytes)
 *   d_ws             workspace of vcfc_encode_workspace_size(n, total) bytes
 *                    where total >= sum of d_line_len
 *   d_err            one uint64: ~0 = success, else (row << 8 | status) of the
 *                    first failing row (rows before it are valid output)
 * Output bytes: [0, d_rec_off[n]) hold the records; with deferred records a
 * call may also write stale bytes into [d_rec_off[n], out_cap) (records
 * placed on predicted offsets before a misprediction is found), never past
 * out_cap -- several batches that share one buffer go in row order.
 * Returns VCFC_OK if the work was enqueued.  Capturable in a hipGraph: the
 * per-call state is reset by a kernel, not by hipMemsetAsync -- on this ROCm
 * a captured 24-byte memset node writes garbage into its first 16 bytes from
 * the second replay on (4- and 8-byte nodes replay correctly;
 * tools/dbg/memset_graph_probe.py, profiles/r04/memset_graph_probe.txt).
 * The n == 0 call enqueues two 8-byte memsets (safe).  The host-driven entry
 * points below (vcfc_compress_*, the decoders) synchronise and are not meant
 * for capture. */
int vcfc_encode_rows_device(const uint8_t *d_buf, const uint64_t *d_line_off,
                            const uint32_t *d_line_len, uint64_t n, uint64_t total_line_bytes,
                            uint8_t *d_out, uint64_t out_cap, uint64_t *d_rec_off,
                            void *d_ws, uint64_t ws_bytes, uint64_t *d_err, void *stream);

/* Rows the last vcfc_encode_rows_device call on workspace d_ws (sized for
 * n, total_line_bytes) deferred and wrote straight into the output (see
 * vcfc_ctx_set_deferred_records; a row whose predicted size led there but
 * whose later bytes sent it to the general path, or that held a '\n' or
 * failed, is not counted); waits for `stream`. */
int vcfc_encode_deferred_rows(const void *d_ws, uint64_t n_rows, uint64_t total_line_bytes, void *stream,
                              uint64_t *rows);

/* Per-stage timing of vcfc_encode_rows_device (HIP events on the same
 * stream).  vcfc_timer_read synchronises and returns the per-stage totals in
 * ms summed over the timed calls since the last read:
 *   ms[0] slot-offset scan, ms[1] k_encode (the fast and variable-token
 *   kernels, plus k_encode_defer's deferred records after the compaction),
 *   ms[2] record-offset scan, ms[3] k_compact;  *calls = number of timed
 *   calls. */
typedef struct vcfc_timer vcfc_timer;
int vcfc_timer_create(vcfc_timer **t);
void vcfc_timer_destroy(vcfc_timer *t);
int vcfc_encode_rows_device_timed(const uint8_t *d_buf, const uint64_t *d_line_off,
                                  const uint32_t *d_line_len, uint64_t n, uint64_t total_line_bytes,
                                  uint8_t *d_out, uint64_t out_cap, uint64_t *d_rec_off,
                                  void *d_ws, uint64_t ws_bytes, uint64_t *d_err, void *stream,
                                  vcfc_timer *t);
int vcfc_timer_read(vcfc_timer *t, double ms[4], uint64_t *calls);

/* Host batch encode (synchronous: H2D, encode on the context's GPU, D2H).
 * rec_off has n + 1 entries.  On a failing row, returns its status and
 * *err_row = its index; records of the rows before it are in `out`. */
int vcfc_encode_rows(vcfc_ctx *ctx, const uint8_t *buf, uint64_t buf_bytes,
                     const uint64_t *line_off, const uint32_t *line_len, uint64_t n,
                     uint8_t *out, uint64_t out_cap, uint64_t *rec_off, int64_t *err_row);

/* ---- whole files: compress() / decompress2_fd() ---------------------------
 * compress: header ("##" and "#") lines pass through with '\n', empty lines
 * are skipped, data lines are encoded on the GPU (reference
 * src/compress.cpp:205-257).  On error returns the status and *err_line =
 * 1-based input line number. */
int vcfc_compress_file(vcfc_ctx *ctx, const char *in_path, const char *out_path, int64_t *err_line);
/* In-memory variant of vcfc_compress_file (out_cap >= vcfc_compress_bound). */
uint64_t vcfc_compress_bound(uint64_t in_bytes);
int vcfc_compress_buffer(vcfc_ctx *ctx, const uint8_t *in, uint64_t n, uint8_t *out, uint64_t out_cap,
                         uint64_t *out_len, int64_t *err_line);

/* compress() over VCF file bytes already resident in device memory (a
 * pipeline stage that produced or received the file on the GPU): d_in[0, n)
 * holds the file's bytes as read, with n > 0 and d_in[n - 1] == '\n' (append
 * one to an unterminated last line: getline returns it, reference
 * src/compress.cpp:218); else VCFC_E_ARG.  The line index and the encoder run
 * on the context's GPU; the bytes compress() writes -- '#' lines verbatim in
 * place, records of the data lines -- land at d_out[0, *out_len) (out_cap >=
 * vcfc_compress_bound(n)).  Runs on the context's stream: complete the
 * writes of d_in first.  Synchronous (the host reads the index counts and
 * the '#' lines).  Statuses and *err_line as vcfc_compress_buffer; on a
 * failing line d_out holds the output of the lines before it. */
int vcfc_compress_device(vcfc_ctx *ctx, const uint8_t *d_in, uint64_t n, uint8_t *d_out, uint64_t out_cap,
                         uint64_t *out_len, int64_t *err_line);

/* One rank's share of a multi-GPU compress (SURVEY §8 e): compresses the
 * byte range [off, off + len) of in_path (whole lines: off at a line start,
 * off + len after a '\n' or at EOF) through the same pipeline and writes the
 * output to out_fd at out_off onwards (pwrite; nothing else in the file is
 * touched).  *out_bytes = bytes written (on a failing line: the output of the
 * lines before it), *err_line = 1-based line within the range, *lines =
 * lines in the range (for global line numbers).  The concatenation of the
 * ranks' outputs in range order equals vcfc_compress_file's output (compress()
 * keeps no state across lines, reference src/compress.cpp:205-257). */
int vcfc_compress_range(vcfc_ctx *ctx, const char *in_path, uint64_t off, uint64_t len, int out_fd,
                        uint64_t out_off, uint64_t *out_bytes, int64_t *err_line, uint64_t *lines);

/* vcfc_compress_range with the output held for a later placement: the
 * rank's offset in the output file is the exclusive prefix of the ranks' byte
 * counts, known only after their all-gather.  The first mem_bound bytes stay
 * in host memory, the rest go to an unlinked temporary file in spill_dir
 * (NULL: /tmp).  vcfc_held_place writes all held bytes at out_off of out_fd
 * (memory blocks by pwrite, the spilled part by copy_file_range), so output
 * that fits in memory is written once, to its final place.  *held is set even
 * on a failing line (it holds the output of the lines before it); free it
 * with vcfc_held_free. */
typedef struct vcfc_held vcfc_held;
int vcfc_compress_range_held(vcfc_ctx *ctx, const char *in_path, uint64_t off, uint64_t len, uint64_t mem_bound,
                             const char *spill_dir, vcfc_held **held, uint64_t *out_bytes, int64_t *err_line,
                             uint64_t *lines);
int vcfc_held_place(const vcfc_held *held, int out_fd, uint64_t out_off);
/* bytes held in host memory / in the spill file */
void vcfc_held_sizes(const vcfc_held *held, uint64_t *mem_bytes, uint64_t *spill_bytes);
void vcfc_held_free(vcfc_held *held);

/* ---- decoder: decompress2_fd (reference src/compress.cpp:1214-1257,
 * decompress2_data_line :741-986) ----------------------------------------
 * .vcfc bytes -> VCF text, byte-identical to the reference's `main
 * decompress`.  The sample count comes from the header line (as in the
 * reference).  On VCFC_E_FORMAT (where the reference throws) the output holds
 * the header and every line the reference writes before throwing.
 * vcfc_decompress_buffer: VCFC_E_NOSPACE if out_cap is short; *out_len is
 * then the size needed. */
int vcfc_decompress_buffer(vcfc_ctx *ctx, const uint8_t *in, uint64_t in_bytes, uint8_t *out, uint64_t out_cap,
                           uint64_t *out_len);
int vcfc_decompress_file(vcfc_ctx *ctx, const char *in_vcfc, const char *out_vcf);

/* Device-resident batch: records d_in[d_rec_start[i], d_rec_start[i+1]) for
 * i < n (e.g. an encoder batch's rec_off), `samples` from the header line.
 * Enqueued on `stream` with no host synchronisation.  Lines land at
 * d_out + d_line_off[i] (n + 1 offsets, d_line_off[n] = total).  d_err:
 * ~0, or min over records of (i << 8 | 2) where a record's byte-serial parse
 * ends off its LEN (the file decoder then continues byte-serially) or
 * (i << 8 | 3) where the reference throws; such records get no line, and
 * lines past the first one are not meaningful.  (i << 8 | 0xFF): out_cap
 * too small.  exact = 0 plans from the headers and REQ bytes only and
 * assumes every sample section is "simple" (3-byte tokens, exactly
 * `samples` of them); the writer checks that and reports (i << 8 | 4) where
 * it was wrong: call again with exact = 1. */
uint64_t vcfc_decode_workspace_size(uint64_t n_records);
int vcfc_decode_records_device(const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_rec_start, uint64_t n,
                               uint64_t samples, uint8_t *d_out, uint64_t out_cap, uint64_t *d_line_off,
                               void *d_ws, uint64_t ws_bytes, uint64_t *d_err, int exact, void *stream);
/* As vcfc_decode_records_device, for the records with d_select[i] != 0 only
 * (the others get no line: d_line_off[i + 1] == d_line_off[i]); d_select =
 * the range query's match flags (vcfc_query_match_device). */
int vcfc_decode_selected_device(const uint8_t *d_in, uint64_t in_bytes, const uint64_t *d_rec_start,
                                const uint8_t *d_select, uint64_t n, uint64_t samples, uint8_t *d_out,
                                uint64_t out_cap, uint64_t *d_line_off, void *d_ws, uint64_t ws_bytes,
                                uint64_t *d_err, int exact, void *stream);

/* ---- range query: query_compressed_file (reference src/main.cpp:3777-3929)
 * Lines (no header) of the records whose CHROM equals `ref` (ref_len == 0:
 * any name) and, when has_range, whose POS lies in [start, end]
 * (VcfCoordinateQuery::matches, src/main.cpp:75-86), byte-identical to the
 * reference's stdout.  On VCFC_E_FORMAT (where the reference throws) the
 * output holds every line the reference writes before throwing.
 * vcfc_parse_query restates parse_coordinate_string (src/main.cpp:3993-4026):
 * "<ref>" or "<ref>:<start>-<end>"; returns 0, or 1 (no '-' after the ':'),
 * 2 (start does not parse), 3 (end does not parse) where the reference
 * prints its message and exits 1; *ref_len = bytes of q holding the name.
 * vcfc_query_buffer: VCFC_E_NOSPACE if out_cap is short (*out_len = size
 * needed); vcfc_query_file writes to out_fd as lines are decoded. */
int vcfc_parse_query(const char *q, uint64_t q_len, uint64_t *ref_len, int *has_range, uint64_t *start,
                     uint64_t *end);
int vcfc_query_buffer(vcfc_ctx *ctx, const uint8_t *in, uint64_t in_bytes, const char *ref, uint64_t ref_len,
                      int has_range, uint64_t start, uint64_t end, uint8_t *out, uint64_t out_cap,
                      uint64_t *out_len);
int vcfc_query_file(vcfc_ctx *ctx, const char *in_vcfc, const char *ref, uint64_t ref_len, int has_range,
                    uint64_t start, uint64_t end, int out_fd);
/* Device-resident match step: d_flag[i] = 1 where record
 * d_in[d_rec_start[i], d_rec_start[i+1]) matches; *d_err = ~0 or min over
 * records of (i << 8 | 2) where its POS does not parse (the reference
 * throws) or (i << 8 | 3) where CHROM/POS runs past the record (the
 * reference's walk leaves the LEN hops there).  d_ref is device memory.
 * Enqueued on `stream`; decode the flagged records with
 * vcfc_decode_selected_device. */
int vcfc_query_match_device(const uint8_t *d_in, const uint64_t *d_rec_start, uint64_t n, const uint8_t *d_ref,
                            uint64_t ref_len, int has_range, uint64_t start, uint64_t end, uint8_t *d_flag,
                            uint64_t *d_err, void *stream);

/* ---- sparse layout: sparsify_file (reference src/sparse.cpp:290-580) -------
 * Record i of the .vcfc goes to data_start + (300e6 + POS_i) * 16384
 * (compute_sparse_offset, src/sparse.cpp:18-51) behind a 16-byte prefix
 * BE(dist_to_prev) BE(dist_to_next); the 8 bytes before data_start hold the
 * first record's offset in host byte order.  Output is a sparse file (holes
 * between records).  The GPU plans offsets and prefixes; the host writes. */
uint64_t vcfc_sparse_offset(uint64_t pos);
int vcfc_sparsify_file(vcfc_ctx *ctx, const char *in_vcfc, const char *out_sparse);
/* Sharded sparsify (multi-GPU, one process per GPU; SURVEY §8 e).  Rank
 * `rank` of `world` owns records [n*rank/world, n*(rank+1)/world) and plans
 * them on its GPU with one halo record on each side (the neighbours' offsets
 * give its first dist_to_prev and last dist_to_next).  info[4] =
 * {lo, hi, first unparsable record (global index, ~0 = none; bytes after the
 * last whole record count as record n), 1 if adjacent records of the planned
 * range overlap or are out of order}.
 * out_sparse == NULL: plan only.  Otherwise the slice is also written into
 * out_sparse (opened without truncation): rank 0 writes the header lines, the
 * owner of record 0 the first-offset slot.  Writing is only valid when every
 * rank's plan reported no error and no anomaly (records then occupy disjoint
 * ranges, so concurrent writes equal the reference's sequential ones);
 * otherwise one rank runs vcfc_sparsify_file, which replays the reference's
 * write order.  VCFC_E_ARG when asked to write a slice whose own plan is not
 * clean. */
int vcfc_sparsify_shard(vcfc_ctx *ctx, const char *in_vcfc, const char *out_sparse, int rank, int world,
                        uint64_t info[4]);
/* Sparse-file query: query_sparse_file_fd (reference src/main.cpp:235-582)
 * over a file written by sparsify, stdout-identical to the reference's
 * `main sparse-query`: start == end looks up the one slot of `start` and
 * writes its line unfiltered; otherwise the lines from the first record at or
 * after start's slot while CHROM equals `ref` and POS <= end (no filter at
 * all: the reference throws).  Lines go to out_fd as they are decoded (on the
 * GPU).  VCFC_E_FORMAT where the reference throws (every line it writes
 * before is written); VCFC_E_IO when the file does not open. */
int vcfc_sparse_query_file(vcfc_ctx *ctx, const char *in_sparse, const char *ref, uint64_t ref_len, int has_range,
                           uint64_t start, uint64_t end, int out_fd);

/* Device plan: records d_recs[d_rec_off[i] .. d_rec_off[i+1]); outputs
 * d_file_off[i] and d_prefix16[16 i ..]; d_status[0] = ~0 or (row << 8 |
 * VCFC_E_FORMAT) of the first record whose POS does not parse, d_status[1] =
 * 1 if records overlap / are out of order (write them in order). */
int vcfc_sparse_plan_device(const uint8_t *d_recs, const uint64_t *d_rec_off, uint64_t n, uint64_t data_start,
                            uint64_t *d_file_off, uint8_t *d_prefix16, uint64_t *d_status, void *stream);

/* ---- device-side helpers used by the benchmark ---------------------------
 * Synthetic genotype rows generated in HBM (no host round trip).  `law`:
 *   0 = random_vcf law (alleles i.i.d. 0/1/2 with p .90/.08/.02,
 *       reference other/random_vcf.py:66-70)
 *   1 = chr22-shaped (per-row alt-allele frequency from d_row_af; ~1% of
 *       rows multi-allelic)
 *   2 = general shapes (d_row_af = kind + allele frequency: haploid,
 *       GT:DP:GQ, missing, unphased; vcf-compression_amd/workload.py)
 *   3 = alternating classes, the RLE worst case (d_row_af = kind: 0 = the
 *       classes 0|0 0|1 1|0 1|1 cycling, every token a new run; 1 = alleles
 *       i.i.d. at frequency 1/2)
 * The prefix (9 columns + '\t') of row i is copied from
 * d_prefix[d_prefix_off[i] .. d_prefix_off[i+1]); row i is written at
 * d_buf + d_line_off[i] with S tokens and a trailing '\n'. */
int vcfc_synth_rows_device(uint8_t *d_buf, const uint64_t *d_line_off, uint64_t n,
                           const uint8_t *d_prefix, const uint64_t *d_prefix_off,
                           const float *d_row_af, uint32_t samples, int law, uint64_t seed,
                           void *stream);
/* The same rows as rows [row_base, row_base + n) of a batch generated whole
 * with this seed (the genotypes hash the batch row index): a rank generates
 * its slice of one fixed dataset (bench.py's strong split). */
int vcfc_synth_rows_device_at(uint8_t *d_buf, const uint64_t *d_line_off, uint64_t n,
                              const uint8_t *d_prefix, const uint64_t *d_prefix_off,
                              const float *d_row_af, uint32_t samples, int law, uint64_t seed,
                              uint64_t row_base, void *stream);

/* Per-record 64-bit digests of an encoded batch, in place on the GPU:
 * d_hash[i] = digest of d_recs[d_rec_off[i] .. d_rec_off[i+1]).  Digest:
 * h = len * 0x9E3779B97F4A7C15 + sum_k mix(w_k ^ (k * 0xD1B54A32D192ED03 +
 * 0x8CB92BA72F3D8DD7)) mod 2^64, result mix(h); w_k = bytes [8k, 8k+8)
 * little-endian, zero-padded; mix = splitmix64's finaliser.  Lets a caller
 * verify multi-GB batches against a CPU encode by comparing 8 B per row (no
 * reference counterpart).  Enqueued on `stream`. */
int vcfc_record_hash_device(const uint8_t *d_recs, const uint64_t *d_rec_off, uint64_t n, uint64_t *d_hash,
                            void *stream);

#ifdef __cplusplus
}
#endif
#endif
