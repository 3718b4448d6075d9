// TEST INFRASTRUCTURE ONLY: the reference-side binding of INTEGRATION.md
// sections 1 and 2, verbatim (tests/test_integration_shim.py checks that
// every line below the marker is the document's code, then compiles this
// file against the reference's own src/compress.hpp / utils.hpp with
// -std=c++11 and links it against build/libvcfc.so).
// ---- INTEGRATION.md ----
// src/compress_gpu_shim.cpp  (added to the reference's SOURCE list)
#include "compress.hpp"
#include "vcfc.h"

static vcfc_ctx *g_vcfc = nullptr;   // one per process / GPU

int compress_data_line(const std::string& line, const VcfCompressionSchema& /*schema: unused, as in the reference*/,
                       std::vector<byte_t>& byte_vec, bool add_newline) {
    if (!g_vcfc && vcfc_ctx_create(0, &g_vcfc) != VCFC_OK)
        throw std::runtime_error("no gfx950 GPU visible");
    const size_t at = byte_vec.size();                  // the reference appends
    byte_vec.resize(at + vcfc_encode_bound(1, line.size()) + 16);
    uint64_t n = 0;
    int st = vcfc_compress_data_line(g_vcfc, line.data(), line.size(), add_newline,
                                     byte_vec.data() + at, byte_vec.size() - at, &n);
    byte_vec.resize(at + (st == VCFC_OK ? n : 0));
    if (st == VCFC_E_LT8COLS) throw VcfValidationError("VCF data line did not contain at least 8 terms");
    if (st == VCFC_E_8COLS) throw std::length_error("vector::_M_default_append");   // reference aborts here
    if (st == VCFC_E_TOOLONG) throw std::length_error(vcfc_strerror(st));           // record past the 30-bit LEN header
    if (st != VCFC_OK) throw std::runtime_error(vcfc_strerror(st));
    return 0;
}

int compress(const std::string& in, const std::string& out) {
    vcfc_ctx *ctx = nullptr;
    if (vcfc_ctx_create(0, &ctx) != VCFC_OK) throw std::runtime_error("no gfx950 GPU visible");
    int64_t line = -1;
    int st = vcfc_compress_file(ctx, in.c_str(), out.c_str(), &line);
    vcfc_ctx_destroy(ctx);
    if (st == VCFC_E_LT8COLS) throw VcfValidationError("VCF data line did not contain at least 8 terms");
    if (st == VCFC_E_HEADER) throw VcfValidationError("VCF Header did not have enough columns");
    if (st == VCFC_E_8COLS) throw std::length_error("vector::_M_default_append");
    if (st == VCFC_E_TOOLONG) throw std::length_error(vcfc_strerror(st));
    if (st != VCFC_OK) throw std::runtime_error(vcfc_strerror(st));
    return 0;
}
