// restart_model.cpp -- TEST HARNESS (CPU): checks the restart planner of the product
// (libmems_amd/csrc/restart_plan.h, the same code the GPU runs) against the literal
// SearchRange restatement of the oracle (oracle/mums_oracle.c).
//
// Model = the GPU path's formulation: per-genome sorted mer lists -> restart plan ->
// records live iff SML index >= start point of their key's phase -> one G-way merge of
// the live records -> default-tolerance groups (MemHash.cpp:139-162) -> HashMatch /
// SetDirection / CalculateOffset probe rows -> the oracle's AddHashEntry replay
// (oracle_replay_rows).  The result must equal oracle_find_matches (literal merge).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../libmems_amd/csrc/restart_plan.h"
#include "../oracle/mums_oracle.h"

using namespace mums::restart;

namespace {
struct Rec {
    uint64_t ck;
    uint32_t g;
    uint32_t pos;
    uint64_t idx;   // SML index in genome g
};
}  // namespace

extern "C" int restart_model_check(int G, const char* const* seqs, const uint64_t* lens, uint64_t seed, int masked,
                                   uint64_t seq_mask, const uint64_t* start_points, uint64_t* stats /* 8 */) {
    if (G < 1 || G > 64) return -1;
    const int L = oracle_seed_length((int64_t)seed), w = oracle_seed_weight((int64_t)seed);
    std::vector<uint64_t> m(G), base(G + 1, 0);
    std::vector<std::vector<uint64_t>> keys(G);
    std::vector<std::vector<uint32_t>> pos(G);
    for (int g = 0; g < G; ++g) {
        m[g] = lens[g] < (uint64_t)L ? 0 : lens[g] - L + 1;
        keys[g].resize(m[g] + 1);
        pos[g].resize(m[g] + 1);
        if (oracle_seed_keys(seqs[g], lens[g], seed, keys[g].data())) return -2;
        if (oracle_build_sml(seqs[g], lens[g], seed, pos[g].data())) return -2;
        base[g + 1] = base[g] + m[g];
    }
    auto ckey_of = [&](uint64_t k) { return ((k >> (64 - 2 * w)) << 1) | (k & 1); };
    std::vector<uint64_t> ck(base[G] + 1);
    std::vector<Rec> all;
    all.reserve(base[G]);
    for (int g = 0; g < G; ++g)
        for (uint64_t i = 0; i < m[g]; ++i) {
            const uint64_t c = ckey_of(keys[g][pos[g][i]]);
            ck[base[g] + i] = c;
            all.push_back(Rec{c, (uint32_t)g, pos[g][i], i});
        }
    std::stable_sort(all.begin(), all.end(), [](const Rec& a, const Rec& b) {
        if (a.ck != b.ck) return a.ck < b.ck;
        return a.g < b.g;
    });
    // candidates: masked keys with more than 1000 records
    std::vector<uint64_t> cand;
    for (size_t i = 0; i < all.size();) {
        size_t j = i;
        while (j < all.size() && (all[j].ck >> 1) == (all[i].ck >> 1)) ++j;
        if (j - i > kRepeatLimit) cand.push_back(all[i].ck >> 1);
        i = j;
    }
    PlanData d{G, m.data(), base.data(), ck.data()};
    const uint64_t C = cand.size();
    std::vector<uint64_t> clo(C * G + 1), chi(C * G + 1), cbp(C * G + 1);
    std::vector<int> cseq(C + 1);
    for (uint64_t c = 0; c < C; ++c)
        cand_precompute(d, cand[c], &clo[c * G], &chi[c * G], &cbp[c * G], &cseq[c]);
    std::vector<uint64_t> S0(G, 0), S(G);
    if (start_points)
        for (int g = 0; g < G; ++g) S0[g] = start_points[g];
    S = S0;
    std::vector<uint64_t> rkey(C + 1), rS((C + 1) * G);
    PlanOut out{};
    out.cap = C + 1;
    out.rkey = rkey.data();
    out.rS = rS.data();
    restart_plan(d, cand.data(), C, clo.data(), chi.data(), cbp.data(), cseq.data(), S.data(), &out);
    // liveness by phase, then groups over the live records
    const uint64_t R = out.nrestarts;
    auto start_of = [&](uint64_t v, int g) {
        const uint64_t p = (uint64_t)(std::upper_bound(rkey.begin(), rkey.begin() + R, v) - rkey.begin());
        return p == 0 ? S0[g] : rS[(p - 1) * G + g];
    };
    std::vector<Rec> live;
    for (const Rec& r : all)
        if (r.idx >= start_of(r.ck >> 1, r.g)) live.push_back(r);
    std::vector<int64_t> rows;
    uint64_t groups = 0;
    for (size_t i = 0; i < live.size();) {
        size_t j = i;
        while (j < live.size() && (live[j].ck >> 1) == (live[i].ck >> 1)) ++j;
        ++groups;
        // MemHash::EnumerateMatches with repeat_tol 0, enum_tol 1: no genome twice
        uint64_t seen = 0;
        bool dup = false;
        for (size_t k = i; k < j; ++k) {
            dup = dup || ((seen >> live[k].g) & 1);
            seen |= 1ull << live[k].g;
        }
        if (j - i >= 2 && !dup) {
            std::vector<int64_t> s(G, 0);
            std::vector<int> par(G, 0);
            for (size_t k = i; k < j; ++k) {
                s[live[k].g] = (int64_t)live[k].pos + 1;
                par[live[k].g] = (int)(live[k].ck & 1);
            }
            int ref = 0;
            while (s[ref] == 0) ++ref;
            for (int g = ref + 1; g < G; ++g)   // SetDirection, MemHash.cpp:189-203
                if (s[g] != 0 && par[g] != par[ref]) s[g] = -s[g];
            int64_t off = 0;
            uint64_t mn = 0;
            for (int g = 0; g < G; ++g) {
                if (g > ref && s[g] != 0) off += s[g] - s[ref] - (s[g] < 0 ? L : 0);
                mn = (mn << 1) | (s[g] != 0 ? 1u : 0u);
            }
            if (!masked || seq_mask == 0 || mn == seq_mask) {
                rows.insert(rows.end(), s.begin(), s.end());
                rows.push_back(off);
            }
        }
        i = j;
    }
    oracle_params prm{};
    prm.seed = seed;
    prm.enum_tol = 1;
    prm.table_size = 40000;
    oracle_result* a = oracle_replay_rows(G, seqs, lens, &prm, rows.data(), rows.size() / (G + 1));
    prm.masked = masked;
    prm.seq_mask = seq_mask;
    prm.start_points = start_points;
    oracle_result* b = oracle_find_matches(G, seqs, lens, &prm);
    if (!a || !b) return -3;
    int rc = 0;
    const uint64_t na = oracle_result_count(a), nb = oracle_result_count(b);
    stats[0] = na;
    stats[1] = nb;
    stats[2] = R;
    stats[3] = oracle_result_restarts(b);
    stats[4] = out.checked;
    stats[5] = out.walk_steps;
    stats[6] = C;
    stats[7] = rows.size() / (G + 1);
    if (na != nb) rc = 1;
    else if (na) {
        std::vector<uint64_t> la(na), lb(na);
        std::vector<int64_t> sa(na * G), sb(na * G);
        oracle_result_copy(a, la.data(), sa.data());
        oracle_result_copy(b, lb.data(), sb.data());
        if (la != lb || sa != sb) rc = 2;
    }
    if (rc == 0 && oracle_result_collision_count(a) != oracle_result_collision_count(b)) rc = 4;
    oracle_result_free(a);
    oracle_result_free(b);
    return rc;
}

// The sharded mode's plan (mums_shard_restart_*): the whole-stream SMLs cut into W key ranges
// of 2^B MSD buckets (balanced counts, shard_comm.hip key_ranges); every rank plans its own
// candidates on its SML parts (PlanData's distributed form: off / n / prv / nxt / key range),
// rank after rank with the running start points.  stats: [restarts whole, restarts
// distributed, undecidable, plans equal, candidates].
extern "C" int restart_model_dist(int G, const char* const* seqs, const uint64_t* lens, uint64_t seed,
                                  const uint64_t* start_points, int W, int B, uint64_t* stats /* 5 */) {
    if (G < 1 || G > 64 || W < 1) return -1;
    const int L = oracle_seed_length((int64_t)seed), w = oracle_seed_weight((int64_t)seed);
    const int kbits = 2 * w + 1;
    if (B < 1 || B > kbits - 1) return -1;
    std::vector<uint64_t> m(G), base(G + 1, 0);
    std::vector<std::vector<uint64_t>> keys(G);
    std::vector<std::vector<uint32_t>> pos(G);
    for (int g = 0; g < G; ++g) {
        m[g] = lens[g] < (uint64_t)L ? 0 : lens[g] - L + 1;
        keys[g].resize(m[g] + 1);
        pos[g].resize(m[g] + 1);
        if (oracle_seed_keys(seqs[g], lens[g], seed, keys[g].data())) return -2;
        if (oracle_build_sml(seqs[g], lens[g], seed, pos[g].data())) return -2;
        base[g + 1] = base[g] + m[g];
    }
    auto ckey_of = [&](uint64_t k) { return ((k >> (64 - 2 * w)) << 1) | (k & 1); };
    std::vector<uint64_t> ck(base[G] + 1);
    for (int g = 0; g < G; ++g)
        for (uint64_t i = 0; i < m[g]; ++i) ck[base[g] + i] = ckey_of(keys[g][pos[g][i]]);
    std::vector<uint64_t> S0(G, 0);
    if (start_points)
        for (int g = 0; g < G; ++g) S0[g] = start_points[g];
    // whole-stream plan
    auto cands_in = [&](uint64_t lo, uint64_t hi) {   // masked keys in [lo, hi) with > 1000 records
        std::vector<uint64_t> all;
        for (uint64_t i = 0; i < base[G]; ++i)
            if (ck[i] >= lo && ck[i] < hi) all.push_back(ck[i] >> 1);
        std::sort(all.begin(), all.end());
        std::vector<uint64_t> c;
        for (size_t i = 0; i < all.size();) {
            size_t j = i;
            while (j < all.size() && all[j] == all[i]) ++j;
            if (j - i > kRepeatLimit) c.push_back(all[i]);
            i = j;
        }
        return c;
    };
    auto plan = [&](const PlanData& d, const std::vector<uint64_t>& cand, std::vector<uint64_t>& S,
                    std::vector<uint64_t>& rkey, std::vector<uint64_t>& rS, unsigned* bad) {
        const uint64_t C = cand.size();
        std::vector<uint64_t> clo(C * G + 1), chi(C * G + 1), cbp(C * G + 1);
        std::vector<int> cseq(C + 1);
        std::vector<unsigned> cbad(C + 1, 0);
        for (uint64_t c = 0; c < C; ++c) {
            PlanData dc = d;
            if (d.off) dc.bad = &cbad[c];
            cand_precompute(dc, cand[c], &clo[c * G], &chi[c * G], &cbp[c * G], &cseq[c]);
        }
        std::vector<uint64_t> rk(C + 1), rs((C + 1) * G);
        PlanOut out{};
        out.cap = C + 1;
        out.rkey = rk.data();
        out.rS = rs.data();
        PlanData dp = d;
        dp.bad = bad;
        restart_plan(dp, cand.data(), C, clo.data(), chi.data(), cbp.data(), cseq.data(), S.data(), &out,
                     d.off ? cbad.data() : nullptr);
        rkey.insert(rkey.end(), rk.begin(), rk.begin() + out.nrestarts);
        rS.insert(rS.end(), rs.begin(), rs.begin() + out.nrestarts * G);
        return C;
    };
    std::vector<uint64_t> rkA, rSA, SA = S0;
    const std::vector<uint64_t> candA = cands_in(0, ~0ull);
    plan(PlanData{G, m.data(), base.data(), ck.data()}, candA, SA, rkA, rSA, nullptr);
    // key ranges over 2^B buckets, balanced like key_ranges
    const int sh = kbits - B;
    const uint64_t nb = 1ull << B;
    std::vector<uint64_t> cum(nb + 1, 0);
    for (uint64_t i = 0; i < base[G]; ++i) cum[(ck[i] >> sh) + 1]++;
    for (uint64_t b = 0; b < nb; ++b) cum[b + 1] += cum[b];
    std::vector<uint64_t> bounds{0};
    for (int r = 1; r < W; ++r) {
        const uint64_t target = (cum[nb] * (uint64_t)r + (uint64_t)W - 1) / (uint64_t)W;
        uint64_t b = (uint64_t)(std::lower_bound(cum.begin(), cum.end(), target) - cum.begin());
        bounds.push_back(std::min(std::max(b, bounds.back()), nb));
    }
    bounds.push_back(nb);
    // every rank's SML parts: genome g's indices with keys in the range are one slice
    std::vector<std::vector<uint64_t>> off(W, std::vector<uint64_t>(G + 1, 0)), cnt(W, std::vector<uint64_t>(G + 1, 0));
    std::vector<uint64_t> klo(W), khi(W);
    for (int r = 0; r < W; ++r) {
        klo[r] = bounds[r] << sh;
        khi[r] = bounds[r + 1] >= nb ? ~0ull : bounds[r + 1] << sh;
        for (int g = 0; g < G; ++g) {
            const uint64_t* a = ck.data() + base[g];
            off[r][g] = (uint64_t)(std::lower_bound(a, a + m[g], klo[r]) - a);
            cnt[r][g] = (uint64_t)(std::lower_bound(a, a + m[g], khi[r]) - a) - off[r][g];
        }
    }
    std::vector<uint64_t> rkB, rSB, S = S0;
    unsigned bad = 0;
    uint64_t Ctot = 0;
    for (int r = 0; r < W; ++r) {
        std::vector<uint64_t> lck, lbase(G + 1, 0), prv(G + 1, 0), nxt(G + 1, ~0ull);
        for (int g = 0; g < G; ++g) {
            lbase[g] = lck.size();
            for (uint64_t i = 0; i < cnt[r][g]; ++i) lck.push_back(ck[base[g] + off[r][g] + i]);
            if (off[r][g] > 0) prv[g] = ck[base[g] + off[r][g] - 1];
            if (off[r][g] + cnt[r][g] < m[g]) nxt[g] = ck[base[g] + off[r][g] + cnt[r][g]];
        }
        lck.push_back(0);
        PlanData d{G, m.data(), lbase.data(), lck.data()};
        d.off = off[r].data();
        d.n = cnt[r].data();
        d.prv = prv.data();
        d.nxt = nxt.data();
        d.key_lo = klo[r];
        d.key_hi = khi[r];
        Ctot += plan(d, cands_in(klo[r], khi[r]), S, rkB, rSB, &bad);
    }
    stats[0] = rkA.size();
    stats[1] = rkB.size();
    stats[2] = bad;
    stats[3] = (rkA == rkB && rSA == rSB && SA == S) ? 1 : 0;
    stats[4] = Ctot;
    return 0;
}
