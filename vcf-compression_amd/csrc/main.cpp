// main.cpp -- CLI with the reference's argv contract (src/main.cpp:4028-4185)
// for the codec path: `main compress|decompress|sparsify <in> <out>` and
// `main query|sparse-query <in> <query>`.  Data lines are
// encoded on the GPU through libvcfc.so.  Error messages mirror the
// reference's exceptions (which terminate the reference process).
#include <cstdio>
#include <cstring>
#include <string>
#include <sys/stat.h>

#include "vcfc.h"

static int usage() {
    fprintf(stderr, "./main [compress|decompress|sparsify] <input_file> <output_file>\n"
                    "./main [query|sparse-query] <input_file> <ref>[:<start>-<end>]\n");
    return 1;
}

static bool file_exists(const char *p) {
    struct stat s;
    return stat(p, &s) == 0;
}

int main(int argc, char **argv) {
    if (argc < 2) return usage();
    std::string action(argv[1]);
    if (action == "compress") {
        if (argc < 4) return usage();
        const bool exists = file_exists(argv[2]);
        if (!exists) printf("Input file does not exist: %s\n", argv[2]);
        if (std::string(argv[2]) == argv[3]) {
            fprintf(stderr, "terminate called after throwing an instance of 'std::runtime_error'\n"
                            "  what():  input and output file are the same\n");
            return 134;
        }
        if (!exists) {   // the reference's ifstream reads nothing: an empty output, exit 0
            FILE *f = fopen(argv[3], "w");
            if (f) fclose(f);
            return 0;
        }
        vcfc_ctx *ctx = nullptr;
        int st = vcfc_ctx_create(0, &ctx);
        if (st != VCFC_OK) {
            fprintf(stderr, "vcfc: %s\n", vcfc_strerror(st));
            return 1;
        }
        int64_t err_line = -1;
        st = vcfc_compress_file(ctx, argv[2], argv[3], &err_line);
        vcfc_ctx_destroy(ctx);
        if (st == VCFC_E_LT8COLS || st == VCFC_E_HEADER) {
            fprintf(stderr, "terminate called after throwing an instance of 'VcfValidationError'\n"
                            "  what():  %s (input line %lld)\n", vcfc_strerror(st), (long long)err_line);
            return 134;
        }
        if (st == VCFC_E_8COLS) {
            fprintf(stderr, "terminate called after throwing an instance of 'std::length_error'\n"
                            "  what():  vector::_M_default_append (input line %lld)\n", (long long)err_line);
            return 134;
        }
        if (st != VCFC_OK) {
            fprintf(stderr, "Error in compression of file: %s\n", vcfc_strerror(st));
            return 1;
        }
        return 0;
    }
    if (action == "decompress") {
        // src/main.cpp:4038-4056 -> decompress2_fd (src/compress.cpp:1214)
        if (argc < 4) return usage();
        if (!file_exists(argv[2])) printf("Input file does not exist: %s\n", argv[2]);
        if (std::string(argv[2]) == argv[3]) {
            fprintf(stderr, "terminate called after throwing an instance of 'std::runtime_error'\n"
                            "  what():  input and output file are the same\n");
            return 134;
        }
        vcfc_ctx *ctx = nullptr;
        int st = vcfc_ctx_create(0, &ctx);
        if (st != VCFC_OK) {
            fprintf(stderr, "vcfc: %s\n", vcfc_strerror(st));
            return 1;
        }
        st = vcfc_decompress_file(ctx, argv[2], argv[3]);
        vcfc_ctx_destroy(ctx);
        if (st == VCFC_E_FORMAT) {
            fprintf(stderr, "terminate called after throwing an instance of 'VcfValidationError'\n"
                            "  what():  %s\n", vcfc_strerror(st));
            return 134;
        }
        if (st != VCFC_OK) {
            fprintf(stderr, "Error in compression of file: %s\n", vcfc_strerror(st));
            return 1;
        }
        return 0;
    }
    if (action == "sparsify") {
        // src/main.cpp:4073-4085
        if (argc < 4) return usage();
        if (std::string(argv[2]) == argv[3]) {
            fprintf(stderr, "terminate called after throwing an instance of 'std::runtime_error'\n"
                            "  what():  input and output file are the same\n");
            return 134;
        }
        if (!file_exists(argv[2])) printf("Input file does not exist: %s\n", argv[2]);
        vcfc_ctx *ctx = nullptr;
        int st = vcfc_ctx_create(0, &ctx);
        if (st != VCFC_OK) {
            fprintf(stderr, "vcfc: %s\n", vcfc_strerror(st));
            return 1;
        }
        st = vcfc_sparsify_file(ctx, argv[2], argv[3]);
        vcfc_ctx_destroy(ctx);
        if (st != VCFC_OK) {
            fprintf(stderr, "terminate called after throwing an instance of 'VcfValidationError'\n"
                            "  what():  %s\n", vcfc_strerror(st));
            return 134;
        }
        return 0;
    }
    if (action == "query" || action == "sparse-query") {
        // src/main.cpp:4057-4069 -> parse_coordinate_string (:3993-4026),
        // query_compressed_file (:3777-3929); src/main.cpp:4086-4096 ->
        // query_sparse_file_fd (:235-582).  Matching lines go to stdout.
        const bool sparse = action == "sparse-query";
        if (argc < 4) return usage();
        if (!sparse && !file_exists(argv[2])) printf("Input file does not exist: %s\n", argv[2]);
        const std::string q(argv[3]);
        uint64_t ref_len = 0, start = 0, end = 0;
        int has_range = 0;
        const int pq = vcfc_parse_query(q.data(), q.size(), &ref_len, &has_range, &start, &end);
        if (pq != 0) {
            const size_t colon = q.find(':'), dash = q.find('-', colon + 1);
            if (pq == 1) printf("Query must contain a dash character: <ref>:<start>-<end>\n");
            else if (pq == 2) printf("Failed to parse int from start position: %s\n", q.substr(colon + 1, dash - colon - 1).c_str());
            else printf("Failed to parse int from end position: %s\n", q.substr(dash + 1).c_str());
            printf("Failed to parse query string: %s\n", q.c_str());
            return 1;
        }
        vcfc_ctx *ctx = nullptr;
        int st = vcfc_ctx_create(0, &ctx);
        if (st != VCFC_OK) {
            fprintf(stderr, "vcfc: %s\n", vcfc_strerror(st));
            return 1;
        }
        fflush(stdout);
        st = sparse ? vcfc_sparse_query_file(ctx, argv[2], q.data(), ref_len, has_range, start, end, 1)
                    : vcfc_query_file(ctx, argv[2], q.data(), ref_len, has_range, start, end, 1);
        vcfc_ctx_destroy(ctx);
        if (st == VCFC_E_IO && sparse) {
            perror("open");
            fprintf(stderr, "terminate called after throwing an instance of 'std::runtime_error'\n"
                            "  what():  Failed to open file: %s\n", argv[2]);
            return 134;
        }
        if (st != VCFC_OK) {
            fprintf(stderr, "terminate called after throwing an instance of 'VcfValidationError'\n"
                            "  what():  %s\n", vcfc_strerror(st));
            return 134;
        }
        return 0;
    }
    std::printf("Unknown action name: %s\n", action.c_str());
    return 0;
}
