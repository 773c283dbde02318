// TEST INFRASTRUCTURE ONLY: MemorySML::Create's sort (MemorySML.cpp:45-60) with the real
// libstdc++ std::sort of this toolchain (the reference builds with the same GCC): a
// vector of {position, mer} records filled in position order (FillDnaSeedSML,
// SortedMerList.cpp:771-783) sorted with the function pointer &bmer_lessthan, which
// compares the mer only (SortedMerList.h:311-314).  The oracle's SortedMerList
// (oracle/std_sort.h restatement, oracle_build_sml) must give the same positions, ties
// included.  Keys come from the oracle's GetDnaSeedMer restatement.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "../oracle/mums_oracle.h"

namespace {
struct bmer {   // SortedMerList.h: gnSeqI position; uint64 mer
    uint64_t position;
    uint64_t mer;
};
bool bmer_lessthan(const bmer& a_v, const bmer& m_v) { return a_v.mer < m_v.mer; }
}  // namespace

// positions of the SML of seq (m = SMLLength entries) into out; returns m or -1
extern "C" int64_t model_sml_positions(const char* seq, uint64_t n, uint64_t seed, uint32_t* out) {
    const int L = oracle_seed_length((int64_t)seed);
    const uint64_t m = n < (uint64_t)L ? 0 : n - L + 1;
    std::vector<uint64_t> keys(m + 1);
    if (oracle_seed_keys(seq, n, seed, keys.data())) return -1;
    std::vector<bmer> sml_array(m);
    for (uint64_t i = 0; i < m; ++i) {
        sml_array[i].position = i;
        sml_array[i].mer = keys[i];
    }
    std::sort(sml_array.begin(), sml_array.end(), &bmer_lessthan);
    for (uint64_t i = 0; i < m; ++i) out[i] = (uint32_t)sml_array[i].position;
    return (int64_t)m;
}
