// cli.cpp — `bmh`, the host program: a from-scratch equivalent of the reference main()
// (main.cpp:415-457) whose three compile-time modes become subcommands:
//
//   bmh compress   <in> <out> [--block-size N] [--gpus G]   (-DCOMPRESS,      main.cpp:439-447)
//   bmh decompress <in> <out> [--host]                      (-DDECOMPRESS,    main.cpp:448-456)
//   bmh full_pipeline [dir]                                 (-DFULL_PIPELINE, main.cpp:416-438)
//
// Invoked through a link named bmh_compress / bmh_decompress / bmh_full_pipeline it takes the
// reference's positional arguments directly. The compress stdout line (main.cpp:319-323,
// 402-413) and the record bytes are the reference's; wrong argument counts print the
// reference's message without a newline and return 1 (main.cpp:440-443).
#include <bmh.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

namespace {

bool read_file(const std::string &name, std::vector<uint8_t> &out)
{
    std::ifstream f(name, std::ios::binary);
    if (!f) return false;
    out.assign(std::istreambuf_iterator<char>(f), {});
    return true;
}

bool write_file(const std::string &name, const uint8_t *p, size_t n)
{
    std::ofstream f(name, std::ios::binary);
    if (!f) return false;
    f.write(reinterpret_cast<const char *>(p), (std::streamsize)n);
    return (bool)f;
}

int die(const std::string &what, int st)
{
    std::cerr << "bmh: " << what << ": " << bmh_status_str(st);
    const char *e = bmh_last_error();
    if (e && *e) std::cerr << " (" << e << ")";
    std::cerr << std::endl;
    return 2;
}

struct Gpus {
    std::vector<bmh_ctx *> ctx;
    ~Gpus()
    {
        for (auto *c : ctx) bmh_ctx_destroy(c);
    }
    int open(int want)
    {
        int n = bmh_device_count();
        if (want <= 0 || want > n) want = n > 0 ? (want <= 0 ? 1 : n) : 0;
        for (int d = 0; d < want; ++d) {
            bmh_ctx *c = nullptr;
            int st = bmh_ctx_create(d, &c);
            if (st != BMH_OK) return st;
            ctx.push_back(c);
        }
        return ctx.empty() ? BMH_ENODEV : BMH_OK;
    }
};

// compress(): main.cpp:300-325 (metrics print order: header size first, then print_metrics)
int do_compress(Gpus &g, const std::string &in, const std::string &outn, uint64_t bs)
{
    std::vector<uint8_t> data;
    if (!read_file(in, data)) {
        std::cerr << "bmh: cannot read " << in << std::endl;
        return 2;
    }
    if (data.empty()) {
        std::cerr << "bmh: empty input (the reference crashes on empty input)" << std::endl;
        return 2;
    }
    std::vector<uint8_t> out(bmh_compress_bound(data.size(), bs));
    uint64_t olen = 0;
    int st = bmh_compress_host_multi(g.ctx.data(), (uint32_t)g.ctx.size(), data.data(), data.size(), bs, out.data(),
                                     out.size(), &olen);
    if (st != BMH_OK) return die("compress", st);
    uint64_t header = 0;
    if (bmh_is_container(out.data(), olen)) {
        uint64_t nb = 0;
        bmh_container_info(out.data(), olen, &nb, nullptr);
        header = 32 + 8 * nb;
        for (uint64_t b = 0; b < nb; ++b) {
            const uint8_t *r;
            uint64_t rl;
            bmh_container_record(out.data(), olen, b, &r, &rl);
            uint64_t t = 0;
            memcpy(&t, r + 16, 8);
            header += 24 + t;
        }
    } else {
        uint64_t t = 0;
        memcpy(&t, out.data() + 16, 8);
        header = 24 + t;
    }
    std::cout << "header size: " << double(header) << " $$ ";
    std::cout << "file_name: " << outn << " $$ initial_data_size: " << data.size()
              << " $$ encoded_file_size: " << olen << " $$ bits_avg: " << (8 * double(olen)) / double(data.size())
              << " $$ compress_rate = " << double(olen) / double(data.size()) << std::endl;
    if (!write_file(outn, out.data(), olen)) {
        std::cerr << "bmh: cannot write " << outn << std::endl;
        return 2;
    }
    return 0;
}

// decompress(): main.cpp:327-345, decoded on the GPU (bmh_decompress_dev on the first context);
// with no context (`--host`) by libbmh's host C++ decoder
int do_decompress(bmh_ctx *ctx, const std::string &in, const std::string &outn)
{
    std::vector<uint8_t> data;
    if (!read_file(in, data)) {
        std::cerr << "bmh: cannot read " << in << std::endl;
        return 2;
    }
    auto dec = [&](uint8_t *out, uint64_t cap, uint64_t *n) {
        return ctx ? bmh_decompress_dev(ctx, data.data(), data.size(), out, cap, n)
                   : bmh_decompress_host(data.data(), data.size(), out, cap, n);
    };
    uint64_t n = 0;
    int st = dec(nullptr, 0, &n);
    if (st != BMH_OK) return die("decompress", st);
    std::vector<uint8_t> out(n);
    st = dec(out.data(), n, &n);
    if (st != BMH_OK) return die("decompress", st);
    if (!write_file(outn, out.data(), n)) {
        std::cerr << "bmh: cannot write " << outn << std::endl;
        return 2;
    }
    return 0;
}

bool same_file(const std::string &a, const std::string &b)
{
    std::vector<uint8_t> x, y;
    return read_file(a, x) && read_file(b, y) && x == y;
}

// FULL_PIPELINE: main.cpp:416-438
int do_full_pipeline(Gpus &g, std::string dir)
{
    if (!dir.empty() && dir.back() != '/') dir += '/';
    const char *files[] = {"bib",    "book1",  "book2", "geo",   "news",  "obj1",  "obj2",
                           "paper1", "paper2", "pic",   "progc", "progl", "progp", "trans"};
    int k = 1, bad = 0;
    for (const char *f : files) {
        std::cout << k++ << "/" << 14 << ' ';
        const std::string in = dir + f, enc = dir + f + ".bzap", dec = dir + f + ".decoded";
        int rc = do_compress(g, in, enc, 0);
        if (rc == 0) rc = do_decompress(g.ctx[0], enc, dec);
        const bool ok = rc == 0 && same_file(in, dec);
        bad += !ok;
        std::cout << (ok ? "success" : "fail") << std::endl;
    }
    return bad ? 1 : 0;
}

int usage()
{
    std::cerr << "usage: bmh compress <in> <out> [--block-size N] [--gpus G]\n"
                 "       bmh decompress <in> <out> [--host]   (--host: the host C++ decoder instead of the GPU)\n"
                 "       bmh full_pipeline [calgarycorpus_dir]\n";
    return 1;
}

}  // namespace

int main(int argc, char **argv)
{
    std::string prog = argv[0];
    const size_t sl = prog.find_last_of('/');
    if (sl != std::string::npos) prog = prog.substr(sl + 1);
    std::string mode;
    std::vector<std::string> args;
    if (prog == "bmh_compress" || prog == "bmh_decompress" || prog == "bmh_full_pipeline") {
        mode = prog.substr(4);
        for (int i = 1; i < argc; ++i) args.push_back(argv[i]);
    } else {
        if (argc < 2) return usage();
        mode = argv[1];
        for (int i = 2; i < argc; ++i) args.push_back(argv[i]);
    }
    uint64_t bs = 0;
    int gpus = 1;
    bool host = false;
    std::vector<std::string> pos;
    for (size_t i = 0; i < args.size(); ++i) {
        if (args[i] == "--block-size" && i + 1 < args.size()) bs = std::stoull(args[++i]);
        else if (args[i] == "--gpus" && i + 1 < args.size()) gpus = std::stoi(args[++i]);
        else if (args[i] == "--host") host = true;
        else pos.push_back(args[i]);
    }
    if (mode == "compress" || mode == "decompress") {
        if (pos.size() != 2) {
            std::cout << "Wrong arguments. Pass only input and output file as parameters";
            return 1;
        }
        if (mode == "decompress" && host) return do_decompress(nullptr, pos[0], pos[1]);
        Gpus g;
        int st = g.open(gpus);
        if (st != BMH_OK) return die("gpu", st);
        if (mode == "decompress") return do_decompress(g.ctx[0], pos[0], pos[1]);
        return do_compress(g, pos[0], pos[1], bs);
    }
    if (mode == "full_pipeline") {
        Gpus g;
        int st = g.open(gpus);
        if (st != BMH_OK) return die("gpu", st);
        return do_full_pipeline(g, pos.empty() ? "calgarycorpus/" : pos[0]);
    }
    return usage();
}
