// TEST INFRASTRUCTURE ONLY: the real libstdc++ std::sort / std::partial_sort of this
// toolchain (the reference builds with the same GCC), against which the oracle's
// restatement of the introsort (oracle/eliminate_overlaps.c) is pinned: same permutation
// of equal keys.  SingleStartComparator (AbstractMatch.h:324-351) = key order, NO_MATCH 0.
#include <algorithm>
#include <cstdint>
#include <vector>

extern "C" void model_std_sort(uint32_t* ids, uint64_t n, const uint64_t* key, int heap_only) {
    std::vector<const uint64_t*> v(n);   // pointers, as MatchList sorts Match*
    for (uint64_t i = 0; i < n; ++i) v[i] = key + ids[i];
    auto cmp = [](const uint64_t* a, const uint64_t* b) { return *a < *b; };
    if (heap_only) std::partial_sort(v.begin(), v.end(), v.end(), cmp);
    else std::sort(v.begin(), v.end(), cmp);
    for (uint64_t i = 0; i < n; ++i) ids[i] = (uint32_t)(v[i] - key);
}

// EliminateOverlaps (Aligner.cpp:62-176) over Match* vectors with the real std::sort, for
// the oracle's C restatement: same control flow over value records {len, starts}.
namespace {
struct M {
    int64_t len;
    std::vector<int64_t> s;
};
int64_t a64(int64_t x) { return x < 0 ? -x : x; }
int mult(const M* m) {
    int k = 0;
    for (int64_t v : m->s) k += v != 0;
    return k;
}
void crop_start(M* m, int64_t a) {
    m->len -= a;
    for (auto& v : m->s)
        if (v > 0) v += a;
}
void crop_end(M* m, int64_t a) {
    m->len -= a;
    for (auto& v : m->s)
        if (v < 0) v -= a;
}
}  // namespace

extern "C" uint64_t model_eliminate_overlaps(int G, uint64_t n, const uint64_t* len, const int64_t* s,
                                             uint64_t* len_out, int64_t* s_out, uint64_t cap) {
    std::vector<M*> ml;
    for (uint64_t i = 0; i < n; ++i) ml.push_back(new M{(int64_t)len[i], std::vector<int64_t>(s + i * G, s + i * G + G)});
    if (ml.size() >= 2) {
        for (int seqI = 0; seqI < G; ++seqI) {
            std::sort(ml.begin(), ml.end(), [seqI](const M* a, const M* b) {
                const int64_t x = a64(a->s[seqI]), y = a64(b->s[seqI]);
                if (x == 0 || y == 0) return y != 0;
                return x < y;
            });
            int64_t matchI = 0, nextI = 0, deleted = 0;
            std::vector<M*> nw;
            for (; matchI != (int64_t)ml.size(); matchI++)
                if (ml[matchI]->s[seqI] != 0) break;
            for (; matchI < (int64_t)ml.size(); matchI++) {
                if (!ml[matchI]) continue;
                for (nextI = matchI + 1; nextI < (int64_t)ml.size(); nextI++) {
                    if (!ml[nextI]) continue;
                    bool del_i = false;
                    const int64_t sI = ml[matchI]->s[seqI], lI = ml[matchI]->len, sJ = ml[nextI]->s[seqI];
                    int64_t diff = a64(sJ) - a64(sI) - lI;
                    if (diff >= 0) break;
                    diff = -diff;
                    M* nm;
                    if (mult(ml[nextI]) > mult(ml[matchI]) ||
                        (mult(ml[nextI]) == mult(ml[matchI]) && ml[nextI]->len > ml[matchI]->len)) {
                        nm = new M(*ml[matchI]);
                        if (diff >= lI) {
                            delete ml[matchI];
                            ml[matchI] = nullptr;
                            matchI--;
                            del_i = true;
                            deleted++;
                        } else if (sI > 0) {
                            crop_end(ml[matchI], diff);
                            crop_start(nm, nm->len - diff);
                        } else {
                            crop_start(ml[matchI], diff);
                            crop_end(nm, nm->len - diff);
                        }
                    } else {
                        nm = new M(*ml[nextI]);
                        if (diff >= ml[nextI]->len) {
                            delete ml[nextI];
                            ml[nextI] = nullptr;
                            deleted++;
                        } else if (sJ > 0) {
                            crop_start(ml[nextI], diff);
                            crop_end(nm, nm->len - diff);
                        } else {
                            crop_end(ml[nextI], diff);
                            crop_start(nm, nm->len - diff);
                        }
                    }
                    nm->s[seqI] = 0;
                    if (mult(nm) > 1 && nm->len > 0) nw.push_back(nm);
                    else delete nm;
                    if (del_i) break;
                }
            }
            if (deleted > 0) {
                std::vector<M*> r;
                for (M* m : ml)
                    if (m) r.push_back(m);
                ml.swap(r);
            }
            ml.insert(ml.end(), nw.begin(), nw.end());
        }
    }
    uint64_t k = 0;
    for (M* m : ml) {
        if (k < cap) {
            len_out[k] = (uint64_t)m->len;
            for (int g = 0; g < G; ++g) s_out[k * G + g] = m->s[g];
        }
        ++k;
        delete m;
    }
    return k;
}
