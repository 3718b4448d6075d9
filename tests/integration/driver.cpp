// TEST INFRASTRUCTURE ONLY: exercises the INTEGRATION.md shim the way the
// reference does.  `driver lines <in.vcf> <out>`: the reference's compress()
// loop body around the section-1 compress_data_line (src/compress.cpp:218-250:
// '#' lines copied with '\n', empty lines skipped, one record per data line);
// `driver file <in.vcf> <out>`: the section-2 compress().  Exit 2 on a
// VcfValidationError, 3 on std::length_error (the reference's abort).
#include <cstdio>
#include <fstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "compress.hpp"

int main(int argc, char **argv) {
    if (argc != 4) return 64;
    const std::string mode(argv[1]);
    try {
        if (mode == "file") return compress(argv[2], argv[3]);
        std::ifstream in(argv[2]);
        std::ofstream out(argv[3], std::ios::binary);
        std::string line;
        std::vector<byte_t> rec;
        VcfCompressionSchema schema;
        while (std::getline(in, line)) {
            if (line.empty()) continue;
            if (line[0] == '#') {
                out << line << "\n";
                continue;
            }
            rec.clear();
            compress_data_line(line, schema, rec, true);
            out.write(reinterpret_cast<const char *>(rec.data()), (std::streamsize)rec.size());
        }
        return 0;
    } catch (const VcfValidationError &) {
        return 2;
    } catch (const std::length_error &) {
        return 3;
    }
}
