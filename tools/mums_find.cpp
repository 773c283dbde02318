// mums_find.cpp -- C++ host driver over include/mums_memhash.hpp (the reference-language
// host path).  Generates the SURVEY Appendix-C synthetic genomes (std::mt19937_64) or reads
// one raw/FASTA sequence per file, runs mums::MemHash / MaskedMemHash on the GPU and prints
// the MatchList text (UngappedLocalAlignment.h:200-206), one match per line.
//   mums_find gen G n weight p [mask]        (mask > 0 selects MaskedMemHash)
//   mums_find files weight f1 f2 ...
//   mums_find sml G n weight p [mask]        the drop-in path of Aligner.cpp:1181-1184 /
//       CreateMemorySMLs (MatchList.h:409-435): HipSML::Create per genome (deferred), then
//       MemHash::FindMatches from ml.sml_table; stderr reports the SMLs materialised (0)
//   mums_find smldump G n weight p g stride  genome g's deferred SML read back: every entry
//       (position, mer) through operator[], then FindMer of every stride-th entry's mer
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <random>
#include <sstream>
#include <string>

#include "mums_memhash.hpp"

static std::vector<std::string> generate(int G, uint64_t n, double p, uint64_t seed) {
    std::mt19937_64 rng(seed);
    const char* acgt = "ACGT";
    std::vector<std::string> g(G);
    g[0].resize(n);
    for (uint64_t i = 0; i < n; ++i) g[0][i] = acgt[rng() & 3];
    for (int k = 1; k < G; ++k) {
        g[k] = g[0];
        for (uint64_t i = 0; i < n; ++i)
            if ((rng() % 1000000) < p * 1e6) g[k][i] = acgt[rng() & 3];
        if (k == 2) {
            std::string r(g[k].rbegin(), g[k].rend());
            for (char& c : r) c = c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : 'A';
            g[k] = r;
        }
    }
    return g;
}

static std::string read_seq(const std::string& path) {
    std::ifstream f(path);
    std::string line, s;
    while (std::getline(f, line)) {
        if (!line.empty() && line[0] == '>') continue;
        for (char c : line)
            if (c != '\n' && c != '\r' && c != ' ') s.push_back(c);
    }
    return s;
}

int main(int argc, char** argv) {
    int gpus = 0;        // --gpus N: ShardedMemHash over devices 0..N-1 (RCCL); --local N: one GPU, N ranks
    bool local = false, slices = false;   // --slices: position slices per rank (else genome blocks)
    if (argc > 2 && (std::string(argv[1]) == "--gpus" || std::string(argv[1]) == "--local")) {
        local = std::string(argv[1]) == "--local";
        gpus = atoi(argv[2]);
        argv += 2;
        argc -= 2;
        if (argc > 1 && std::string(argv[1]) == "--slices") {
            slices = true;
            ++argv;
            --argc;
        }
    }
    uint64_t compat_chunk = 0;   // --compat CHUNK: ParallelMemHash (CHUNK_SIZE = CHUNK)
    if (argc > 2 && std::string(argv[1]) == "--compat") {
        compat_chunk = strtoull(argv[2], nullptr, 10);
        argv += 2;
        argc -= 2;
    }
    if (argc < 3) {
        std::cerr << "usage: mums_find [--gpus N | --local N] [--slices] [--compat CHUNK] gen G n weight p [mask] | "
                     "files weight f1 f2 ...\n";
        return 2;
    }
    std::string mode = argv[1];
    if ((mode == "sml" || mode == "smldump") && argc >= 6) {
        const int G = atoi(argv[2]);
        const uint64_t n = strtoull(argv[3], nullptr, 10);
        const int weight = atoi(argv[4]);
        const double p = atof(argv[5]);
        try {
            mums::MatchList ml;
            ml.seq_table = generate(G, n, p, 12345);
            auto t0 = std::chrono::steady_clock::now();
            ml.CreateMemorySMLs((uint32_t)weight);   // Create per genome: no keys, no sort
            auto t1 = std::chrono::steady_clock::now();
            if (mode == "smldump") {
                const uint32_t g = argc > 6 ? (uint32_t)atoi(argv[6]) : 0;
                const uint64_t stride = argc > 7 ? strtoull(argv[7], nullptr, 10) : 1000;
                mums::HipSML& sml = *ml.sml_table.at(g);
                std::ostringstream os;
                const uint64_t m = sml.SMLLength();
                for (uint64_t i = 0; i < m; ++i) {
                    const mums::bmer b = sml[i];
                    os << b.position << '\t' << b.mer << '\n';
                }
                for (uint64_t i = 0; i < m; i += stride) {   // FindMer (SortedMerList.cpp:170-179)
                    uint64_t r = 0;
                    const bool f = sml.FindMer(sml[i].mer, r);
                    os << "find\t" << i << '\t' << f << '\t' << r << '\n';
                }
                std::vector<mums::bmer> rv;   // MemorySML::Read past the end returns false
                const bool ok = sml.Read(rv, 10, m > 5 ? m - 5 : 0);
                os << "read\t" << ok << '\t' << rv.size() << '\n';
                std::cout << os.str();
                std::cerr << "sml length " << m << " materialized " << mums::HipSML::Materializations() << "\n";
                return 0;
            }
            mums::MaskedMemHash mh(0);
            const uint64_t mask = argc > 6 ? strtoull(argv[6], nullptr, 0) : 0;
            if (mask) mh.SetMask(mask);
            else mums_set_mask(mh.handle(), 0, 0);
            mh.FindMatches(ml);   // genomes and seed pattern from ml.sml_table
            auto t2 = std::chrono::steady_clock::now();
            std::ostringstream os;
            for (const auto& m : ml) os << m << '\n';
            std::cout << os.str();
            std::cerr << "matches " << ml.size() << " create ms "
                      << std::chrono::duration<double, std::milli>(t1 - t0).count() << " find ms "
                      << std::chrono::duration<double, std::milli>(t2 - t1).count() << " materialized "
                      << mums::HipSML::Materializations() << "\n";
        } catch (const std::exception& e) {
            std::cerr << "error: " << e.what() << "\n";
            return 1;
        }
        return 0;
    }
    std::vector<std::string> seqs;
    int weight = 0;
    uint64_t mask = 0;
    if (mode == "gen") {
        int G = atoi(argv[2]);
        uint64_t n = strtoull(argv[3], nullptr, 10);
        weight = atoi(argv[4]);
        double p = atof(argv[5]);
        if (argc > 6) mask = strtoull(argv[6], nullptr, 0);
        seqs = generate(G, n, p, 12345);
    } else {
        weight = atoi(argv[2]);
        for (int i = 3; i < argc; ++i) seqs.push_back(read_seq(argv[i]));
    }
    if (gpus > 0) {
        try {
            std::vector<int> devs(gpus, 0);
            for (int r = 0; r < gpus; ++r) devs[r] = local ? 0 : r;
            // RCCL prints its version banner on stdout during communicator setup: keep the
            // MatchList alone on stdout
            std::fflush(stdout);
            const int saved = dup(1);
            dup2(2, 1);
            mums::ShardedMemHash sh(devs, local, slices);
            std::fflush(stdout);
            dup2(saved, 1);
            close(saved);
            sh.SetSeed(weight ? (uint64_t)mums_get_seed(weight, 0) : 0);
            if (compat_chunk) sh.SetParallelCompat(true, compat_chunk);
            for (const auto& s : seqs) sh.AddSequence(s);
            mums::MatchList ml;
            auto t0 = std::chrono::steady_clock::now();
            sh.FindMatches(ml);
            auto t1 = std::chrono::steady_clock::now();
            std::ostringstream os;
            for (const auto& m : ml) os << m << '\n';
            std::cout << os.str();
            std::cerr << "matches " << ml.size() << " ranks " << gpus << " ms "
                      << std::chrono::duration<double, std::milli>(t1 - t0).count() << "\n";
        } catch (const std::exception& e) {
            std::cerr << "error: " << e.what() << "\n";
            return 1;
        }
        return 0;
    }
    try {
        mums::MaskedMemHash mh(0);   // mask 0 behaves exactly like MemHash
        if (compat_chunk && mums_set_parallel_compat(mh.handle(), 1, compat_chunk) != MUMS_OK)
            throw mums::InvalidData(mums_last_error(mh.handle()));
        if (mask) mh.SetMask(mask);
        else mums_set_mask(mh.handle(), 0, 0);
        mh.SetSeed(weight ? (uint64_t)mums_get_seed(weight, 0) : 0);
        mums::MatchList ml;
        ml.seq_table = seqs;
        auto t0 = std::chrono::steady_clock::now();
        mh.FindMatches(ml);
        auto t1 = std::chrono::steady_clock::now();
        std::ostringstream os;
        for (const auto& m : ml) os << m << '\n';
        std::cout << os.str();
        auto st = mh.stats();
        std::cerr << "matches " << ml.size() << " collisions " << st.collision_count << " ms "
                  << std::chrono::duration<double, std::milli>(t1 - t0).count() << "\n";
    } catch (const std::exception& e) {
        std::cerr << "error: " << e.what() << "\n";
        return 1;
    }
    return 0;
}
