/* vcfc_oracle.h -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference
 * codec used as the parity checker (see vcfc_oracle.c header). */
#ifndef VCFC_ORACLE_H
#define VCFC_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* status codes: same values as include/vcfc.h */
#define VCFO_OK 0
#define VCFO_E_LT8COLS 1
#define VCFO_E_8COLS 2
#define VCFO_E_HEADER 3
#define VCFO_E_NOSPACE 4
#define VCFO_E_FORMAT 8
#define VCFO_E_IO 9

int vcfo_encode_line(const uint8_t *line, size_t len, int add_newline,
                     uint8_t *out, size_t cap, size_t *out_len);
size_t vcfo_encode_bound(size_t line_len);
int vcfo_compress(const uint8_t *in, size_t n, uint8_t *out, size_t cap,
                  size_t *out_len, int64_t *err_line);
int vcfo_decompress(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *out_len);
int vcfo_parse_query(const uint8_t *q, size_t n, size_t *ref_len, int *has_range, uint64_t *start, uint64_t *end);
int vcfo_query(const uint8_t *in, size_t n, const uint8_t *qref, size_t qref_len, int has_range,
               uint64_t qstart, uint64_t qend, uint8_t *out, size_t cap, size_t *out_len);
uint64_t vcfo_sparse_offset(uint64_t pos);
int vcfo_sparsify(const uint8_t *in, size_t n, const char *out_path);
int vcfo_sparse_query(const char *path, const uint8_t *qref, size_t qref_len, int has_range, uint64_t qstart,
                      uint64_t qend, uint8_t *out, size_t cap, size_t *out_len);
int vcfo_strtoul_whole(const uint8_t *s, size_t n, uint64_t *out);
/* batch checker: record digest (= vcfc_record_hash_device) and a threaded
 * encode returning per-row status / record size / digest */
uint64_t vcfo_hash64(const uint8_t *p, size_t n);
int vcfo_encode_rows_hash(const uint8_t *buf, const uint64_t *off, const uint32_t *len, uint64_t n, int threads,
                          uint64_t *hash, uint32_t *size, int32_t *status);
#ifdef __cplusplus
}
#endif
#endif
