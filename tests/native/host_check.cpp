// Host code of the drop-in front end without a GPU, for the sanitizer builds
// (tests/test_sanitize.py, `make sanitize`): the CLI's argument parser and
// file loader (kb2e_amd/csrc/host/kb2e_cli.cpp, the reference's
// common/args.cpp:53-122 and common/loader.cpp:15-62) and the host triple
// store + sample stream (kb2e_amd/csrc/host_data.hpp, common/trainer.cpp:79-98).
//   host_check args <flags...>                 the parsed options, one line
//   host_check load <datadir>                  |E| |R| |train| and an id checksum
//   host_check stream <datadir> <seed> <count> <method>
//                                              the first <count> samples "i j side"
#define KB2E_CLI_NO_MAIN
#include "../../kb2e_amd/csrc/host/kb2e_cli.cpp"
#include "../../kb2e_amd/csrc/host_data.hpp"

using namespace kb2e_host;

static void load(const std::string& dir, int& ne, int& nr, std::vector<int32_t>& H, std::vector<int32_t>& T,
                 std::vector<int32_t>& R) {
    std::map<std::string, int> ent, rel;
    loadIdFile(dir + "/entity2id.txt", ent);
    loadIdFile(dir + "/relation2id.txt", rel);
    ne = (int)ent.size();
    nr = (int)rel.size();
    loadTripleFile(dir + "/train.txt", ent, rel, [&](int h, int t, int r) {
        H.push_back(h);
        T.push_back(t);
        R.push_back(r);
    });
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const std::string mode = argv[1];
    if (mode == "args") {
        EmbeddingArguments a = parseArgs(argc - 1, argv + 1);
        printf("%s precision %d device %d transrcompat %d schedule %d gpus %d\n", a.to_string().c_str(), a.precision,
               a.device, a.transrCompat, a.schedule, a.gpus);
        return 0;
    }
    if (argc < 3) return 2;
    int ne = 0, nr = 0;
    std::vector<int32_t> H, T, R;
    load(argv[2], ne, nr, H, T, R);
    if (mode == "load") {
        unsigned long long sum = 0;
        for (size_t k = 0; k < H.size(); ++k) sum = sum * 1000003ull + (unsigned)(H[k] * 31 + T[k] * 7 + R[k]);
        printf("%d %d %zu %llu\n", ne, nr, H.size(), sum);
        return 0;
    }
    if (mode == "stream" && argc >= 6) {
        kb2e::TripleStore ts;
        ts.build(H.data(), T.data(), R.data(), (int64_t)H.size(), ne, nr);
        kb2e::GlibcRand g((uint32_t)atoi(argv[3]));
        const int count = atoi(argv[4]), method = atoi(argv[5]);
        for (int k = 0; k < count; ++k) {
            int32_t si, sj;
            uint8_t side;
            if (!kb2e::HostSampler::draw(g, ts, method, si, sj, side)) return 3;
            printf("%d %d %d\n", si, sj, (int)side);
        }
        return 0;
    }
    return 2;
}
