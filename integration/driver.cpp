// integration/driver.cpp — test harness for integration/compress_bmh.cpp: a main() with the
// argument contract of the reference's COMPRESS / DECOMPRESS builds (main.cpp:439-456) and
// print_metrics with its output format (main.cpp:402-413), standing in for the rest of the
// reference's main.cpp (which a maintainer keeps as it is). Mode: argv[0] ending in
// "decompress" decodes, anything else encodes.
#include <cstring>
#include <iostream>
#include <string>

void compress(const std::string &initial_file_name, const std::string &encoded_file_name);
void decompress(const std::string &encoded_file_name, const std::string &decoded_file_name);

void print_metrics(const std::string &output_file, const size_t &initial_data_size, const size_t &encoded_data_size)
{
    std::cout << "file_name: " << output_file << " $$ initial_data_size: " << initial_data_size
              << " $$ encoded_file_size: " << encoded_data_size
              << " $$ bits_avg: " << (8 * double(encoded_data_size)) / double(initial_data_size)
              << " $$ compress_rate = " << double(encoded_data_size) / double(initial_data_size) << std::endl;
}

int main(int argc, char *argv[])
{
    if (argc != 3) {
        std::cout << "Wrong arguments. Pass only input and output file as parameters";
        return 1;
    }
    const std::string self = argv[0];
    const bool dec = self.size() >= 10 && self.compare(self.size() - 10, 10, "decompress") == 0;
    try {
        if (dec) decompress(argv[1], argv[2]);
        else compress(argv[1], argv[2]);
    } catch (const std::exception &e) {
        std::cerr << "libbmh: " << e.what() << "\n";
        return 2;
    }
    return 0;
}
