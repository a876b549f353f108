// Host check: the device introsort emulation (mam3slam_amd/csrc/introsort.hpp) reproduces libstdc++
// std::sort's output order, ties included, and so does its data-parallel formulation (stl_sort_model), on tie-heavy random inputs of every size 0..600.
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
#include "../../mam3slam_amd/csrc/introsort.hpp"

int main() {
    std::mt19937 rng(1234);
    long checked = 0;
    for (int trial = 0; trial < 40; trial++) {
        for (int n = 0; n <= 600; n += (n < 64 ? 1 : 7)) {
            int nkeys = 1 + (int)(rng() % (trial % 5 == 0 ? 3 : (trial % 5 == 1 ? 20 : 1000)));
            std::vector<std::pair<uint32_t, uint32_t>> ref(n);
            std::vector<mam::SortEl> emu(n);
            for (int i = 0; i < n; i++) {
                uint32_t k = rng() % nkeys;
                if (trial % 7 == 3) k = (uint32_t)(n - i) / 3;      // descending runs
                if (trial % 7 == 4) k = (uint32_t)i / 5;            // ascending runs
                ref[i] = {k, (uint32_t)i};
                emu[i] = {k, (uint32_t)i};
            }
            std::sort(ref.begin(), ref.end(),
                      [](const std::pair<uint32_t, uint32_t>& a, const std::pair<uint32_t, uint32_t>& b) {
                          return a.first < b.first;
                      });
            std::vector<mam::SortEl> par(emu), leaf(emu);
            mam::stl_sort(emu.data(), emu.data() + n);
            mam::stl_sort_model(par.data(), n);   // data-parallel formulation (device wave sort)
            mam::stl_sort_model_leaf(leaf.data(), n);   // ... with the per-leaf final stage (stl_sort_wave2)
            for (int i = 0; i < n; i++) {
                if (ref[i].first != emu[i].key || ref[i].second != emu[i].val) {
                    printf("MISMATCH trial=%d n=%d i=%d\n", trial, n, i);
                    return 1;
                }
                if (ref[i].first != par[i].key || ref[i].second != par[i].val) {
                    printf("MODEL MISMATCH trial=%d n=%d i=%d\n", trial, n, i);
                    return 1;
                }
                if (ref[i].first != leaf[i].key || ref[i].second != leaf[i].val) {
                    printf("LEAF MODEL MISMATCH trial=%d n=%d i=%d\n", trial, n, i);
                    return 1;
                }
            }
            checked++;
        }
    }
    printf("OK %ld arrays\n", checked);
    return 0;
}
