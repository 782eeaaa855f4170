// integration/compress_bmh.cpp — the reference's compress() and decompress() (main.cpp:300-345)
// rewritten against libbmh's C ABI (include/bmh.h). This is what a maintainer puts in main.cpp
// in place of those two functions; everything they call besides libbmh is the reference's own:
//   read_bytes  (io_utilities.h:29-55)  the tuple form, read_meta = false: the whole file
//   write_bytes (io_utilities.h:7-27)   with its SIZE_MAX defaults: raw bytes, no header
//   print_metrics (main.cpp:294-298, 402-413), 3 arguments, after the "header size:" print
//   (main.cpp:319-321), so stdout and the record are byte-identical to the reference's.
// It compiles against the reference's headers as they lie:
//   g++ -std=c++2b -include climits -I /root/reference -I include -c integration/compress_bmh.cpp
// (tests/test_integration.py builds it with integration/driver.cpp and runs it.)
#include <cstdint>
#include <iostream>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "bmh.h"
#include "io_utilities.h"

// the reference's declaration (main.cpp:294-298); its definition stays in main.cpp (:402-413)
void print_metrics(const std::string &output_file, const size_t &initial_data, const size_t &encoded_data_size);

namespace {
// one libbmh context for the process (one per GPU; compress() is called once per file)
bmh_ctx *bmh_context()
{
    static bmh_ctx *ctx = nullptr;
    if (!ctx && bmh_ctx_create(0, &ctx) != BMH_OK) throw std::runtime_error(bmh_last_error());
    return ctx;
}
}  // namespace

void compress(const std::string &initial_file_name, const std::string &encoded_file_name)
{
    const auto &[bytes_input, dummy1, dummy2, dummy3] = read_bytes(initial_file_name);
    // bwt -> move_to_front -> huffman -> tree_to_bytes (main.cpp:305-318) on the GPU, block
    // size 0 = the whole file is one block: the output is the reference's record
    // [u64 primary][u64 n][u64 tree_len][tree][payload] (io_utilities.h:16-25)
    std::vector<unsigned char> record(bmh_compress_bound(bytes_input.size(), 0));
    uint64_t record_len = 0;
    if (bmh_compress_host(bmh_context(), bytes_input.data(), bytes_input.size(), 0, record.data(), record.size(),
                          &record_len) != BMH_OK)
        throw std::runtime_error(bmh_last_error());
    record.resize(record_len);
    const uint64_t size_of_tree = *reinterpret_cast<const uint64_t *>(record.data() + 2 * sizeof(size_t));

    size_t encoded_data_size = sizeof(unsigned char) * size_of_tree;
    encoded_data_size += 2 * sizeof(size_t) + sizeof(unsigned long);
    std::cout << "header size: " << double(encoded_data_size) << " $$ ";
    encoded_data_size = record.size();
    print_metrics(encoded_file_name, bytes_input.size(), encoded_data_size);
    write_bytes(encoded_file_name, record);  // the record already holds its header
}

void decompress(const std::string &encoded_file_name, const std::string &decoded_file_name)
{
    const auto &[record, dummy1, dummy2, dummy3] = read_bytes(encoded_file_name);
    // bytes_to_tree -> huffman_reverse -> move_to_front_reverse -> bwt_reverse (main.cpp:331-342)
    // on the GPU (bmh_decompress_dev: record H2D, the decode kernels, the block D2H); the first
    // call (out = NULL) reads only the size from the header
    uint64_t n = 0;
    if (bmh_decompress_dev(bmh_context(), record.data(), record.size(), nullptr, 0, &n) != BMH_OK)
        throw std::runtime_error(bmh_last_error());
    std::vector<unsigned char> decoded_data(n);
    if (bmh_decompress_dev(bmh_context(), record.data(), record.size(), decoded_data.data(), n, &n) != BMH_OK)
        throw std::runtime_error(bmh_last_error());
    write_bytes(decoded_file_name, decoded_data);
}
