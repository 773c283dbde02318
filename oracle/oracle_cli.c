/*
 * oracle_cli.c -- TEST INFRASTRUCTURE ONLY.
 * Generates an Appendix-C synthetic input, runs the oracle MemHash and prints
 * the MatchList text (`len\ts0\t...\tsG-1`, UngappedLocalAlignment.h:200-206)
 * on stdout; counters go to stderr.
 *   usage: oracle_cli G n weight p [masked(0/1) [mask [rng_seed]]]
 */
#include "mums_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

int main(int argc, char** argv) {
    if (argc < 5) { fprintf(stderr, "usage: %s G n weight p [masked mask rng_seed]\n", argv[0]); return 2; }
    int G = atoi(argv[1]);
    uint64_t n = strtoull(argv[2], 0, 10);
    int w = atoi(argv[3]);
    double p = atof(argv[4]);
    int masked = argc > 5 ? atoi(argv[5]) : 0;
    uint64_t mask = argc > 6 ? strtoull(argv[6], 0, 0) : 0;
    uint64_t rs = argc > 7 ? strtoull(argv[7], 0, 10) : 12345;
    char* buf = (char*)malloc((size_t)G * n);
    oracle_generate(G, n, p, rs, buf);
    const char* seqs[64]; uint64_t lens[64];
    for (int g = 0; g < G; ++g) { seqs[g] = buf + (uint64_t)g * n; lens[g] = n; }
    oracle_params prm = {0};
    prm.seed = (uint64_t)oracle_get_seed(w, 0);
    prm.repeat_tol = 0; prm.enum_tol = 1; prm.table_size = 40000;
    prm.masked = masked; prm.seq_mask = mask;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    oracle_result* r = oracle_find_matches(G, seqs, lens, &prm);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    uint64_t c = oracle_result_count(r);
    uint64_t* L = (uint64_t*)malloc((c + 1) * sizeof(uint64_t));
    int64_t* S = (int64_t*)malloc((c + 1) * G * sizeof(int64_t));
    oracle_result_copy(r, L, S);
    for (uint64_t i = 0; i < c; ++i) {
        printf("%llu", (unsigned long long)L[i]);
        for (int g = 0; g < G; ++g) printf("\t%lld", (long long)S[i * G + g]);
        printf("\n");
    }
    fprintf(stderr, "matches %llu collisions %llu probes %llu max_group %llu seedmers %llu time %.3f s\n",
            (unsigned long long)c, (unsigned long long)oracle_result_collision_count(r),
            (unsigned long long)oracle_result_probe_count(r), (unsigned long long)oracle_result_max_group(r),
            (unsigned long long)oracle_result_seedmers(r),
            (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec));
    oracle_result_free(r);
    free(buf); free(L); free(S);
    return 0;
}
