// Host model of k_distribute2 (mam3slam_amd/csrc/distribute.hpp) for one level: the kernel's phases run one after
// another (a phase's atomics and scans are order-independent sums / prefix sums), the same tables, ranks, creation and
// kept bases, expansion cut and key remapping, the final-phase sort by the libstdc++ introsort emulation the device
// wave sort is checked against (tests/cpp/test_introsort.cpp). tests/test_distribute_model.py compares it with the
// oracle's DistributeOctTree (std::list + std::sort, ORBextractor.cc:555-779): a check of the kernel's algorithm on the
// CPU, independent of the GPU parity tests.
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../mam3slam_amd/csrc/introsort.hpp"

namespace {

struct Rect {
    uint32_t x, y;   // x0 | y0 << 16, x1 | y1 << 16
};

Rect child_rect(Rect r, int q) {
    const int x0 = r.x & 0xFFFF, y0 = r.x >> 16, x1 = r.y & 0xFFFF, y1 = r.y >> 16;
    const int hx = (x1 - x0 + 1) >> 1, hy = (y1 - y0 + 1) >> 1;
    const int cx0 = (q & 1) ? x0 + hx : x0, cx1 = (q & 1) ? x1 : x0 + hx;
    const int cy0 = (q & 2) ? y0 + hy : y0, cy1 = (q & 2) ? y1 : y0 + hy;
    return {(uint32_t)cx0 | ((uint32_t)cy0 << 16), (uint32_t)cx1 | ((uint32_t)cy1 << 16)};
}

int quad(Rect r, uint32_t key) {
    const int x = key & 0xFFF, y = (key >> 12) & 0xFFF;
    const int x0 = r.x & 0xFFFF, y0 = r.x >> 16, x1 = r.y & 0xFFFF, y1 = r.y >> 16;
    const bool right = x >= x0 + ((x1 - x0 + 1) >> 1), bottom = y >= y0 + ((y1 - y0 + 1) >> 1);
    return (right ? 1 : 0) | (bottom ? 2 : 0);
}

struct Table {
    std::vector<Rect> rect;
    std::vector<uint32_t> cnt;
    std::vector<int> xr;
    std::vector<uint32_t> ch;   // 4 per node
};

}  // namespace

// cand: packed x | y << 12 | score << 24 relative to (minX, minY); out: the kept keys in list order. Returns the count,
// -1 on the kernel's overflow conditions.
extern "C" int dist2_model(const uint32_t* cand, int n, int minX, int maxX, int minY, int maxY, int N, uint32_t* out,
                           int cap) {
    if (n == 0) return 0;
    const int nini = (int)roundf((float)(maxX - minX) / (maxY - minY));
    const float hX = (float)(maxX - minX) / nini;
    const int H = maxY - minY;
    const int NC = (N + 3 > 4 * nini ? N + 3 : 4 * nini) + 8 + 4 * n;   // generous: the model checks no capacity
    std::vector<uint32_t> key(cand, cand + n), kn(n, 0);
    Table T[2];
    for (auto& t : T) {
        t.rect.assign(NC, {0, 0});
        t.cnt.assign(NC, 0);
        t.xr.assign(NC, -1);
        t.ch.assign(4 * (size_t)NC, 0);
    }
    std::vector<uint32_t> nb(NC, 0), candl(NC, 0), srt(NC, 0);
    // initial nodes in table 1, compacted into table 0
    for (int i = 0; i < nini; i++) {
        T[1].rect[i] = {(uint32_t)(int)(hX * (float)i), (uint32_t)(int)(hX * (float)(i + 1)) | ((uint32_t)H << 16)};
        T[1].cnt[i] = 0;
    }
    for (int k = 0; k < n; k++) {
        const int i = (int)((float)(key[k] & 0xFFF) / hX);
        kn[k] = (uint32_t)i;
        T[1].cnt[i]++;
    }
    int S = 0;
    for (int i = 0; i < nini; i++) {
        const uint32_t c = T[1].cnt[i];
        if (c > 0) {
            const int np = S++;
            T[0].rect[np] = T[1].rect[i];
            T[0].cnt[np] = c;
            T[0].xr[np] = c > 1 ? 0 : -1;
            for (int q = 0; q < 4; q++) T[0].ch[4 * np + q] = 0;
            nb[i] = (uint32_t)np;
        }
    }
    for (int k = 0; k < n; k++) kn[k] = nb[kn[k]];
    int cur = 0, m = 0;
    bool final_phase = false;
    for (int guard = 0;; guard++) {
        if (guard > 4096) return -1;
        Table& A = T[cur];
        Table& B = T[cur ^ 1];
        if (final_phase && m == 0) break;
        for (int k = 0; k < n; k++) {   // count
            const int p = kn[k] & 0xFFFF;
            if (A.xr[p] >= 0) {
                const int q = quad(A.rect[p], key[k]);
                A.ch[4 * p + q]++;
                kn[k] = (uint32_t)p | ((uint32_t)q << 16);
            }
        }
        auto eb = [&](int p) {
            uint32_t e = 0, b = 0;
            for (int q = 0; q < 4; q++) {
                e += A.ch[4 * p + q] > 0;
                b += A.ch[4 * p + q] > 1;
            }
            return e | (b << 16);
        };
        uint32_t C = 0, M = 0;
        if (final_phase) {
            std::vector<mam::SortEl> arr(m);
            for (int i = 0; i < m; i++) {
                const int p = (int)candl[i];
                arr[i].key = (A.cnt[p] << 12) | (A.rect[p].x & 0xFFFFu);
                arr[i].val = (uint32_t)p;
            }
            mam::stl_sort(arr.data(), arr.data() + m);
            for (int i = 0; i < m; i++) srt[m - 1 - i] = arr[i].val;
            uint32_t pc = 0;
            bool found = false;
            for (int r = 0; r < m; r++) {
                const int p = (int)srt[r];
                const uint32_t v = eb(p);
                const uint32_t incl = pc + v;
                if (found) {
                    A.xr[p] = -1;
                } else {
                    nb[p] = incl - v;
                    if (S + (int)(incl & 0xFFFF) - (r + 1) >= N) {
                        found = true;
                        C = incl & 0xFFFF;
                        M = incl >> 16;
                    }
                }
                pc = incl;
            }
            if (!found) { C = pc & 0xFFFF; M = pc >> 16; }
        }
        uint32_t c1 = 0, c2 = 0;
        for (int p = 0; p < S; p++) {
            const bool ex = A.xr[p] >= 0;
            const uint32_t v1 = (ex && !final_phase) ? eb(p) : 0u, v2 = ex ? 0u : 1u;
            if (!ex) nb[p] = c2;
            else if (!final_phase) nb[p] = c1;
            c1 += v1;
            c2 += v2;
        }
        if (!final_phase) { C = c1 & 0xFFFF; M = c1 >> 16; }
        const uint32_t K = c2;
        const int Snew = (int)(C + K);
        const bool fin = Snew >= N || Snew == S;
        const bool next_final = !fin && (final_phase || Snew + 3 * (int)M > N);
        for (int p = 0; p < S; p++) {
            if (A.xr[p] >= 0) {
                const int cb = nb[p] & 0xFFFF, bb = nb[p] >> 16;
                int j = 0, jb = 0;
                for (int q = 0; q < 4; q++) {
                    const uint32_t cq = A.ch[4 * p + q];
                    if (cq > 0) {
                        const int np = (int)C - 1 - (cb + j);
                        B.rect[np] = child_rect(A.rect[p], q);
                        B.cnt[np] = cq;
                        B.xr[np] = cq > 1 ? 0 : -1;
                        for (int u = 0; u < 4; u++) B.ch[4 * np + u] = 0;
                        if (cq > 1) candl[bb + jb++] = (uint32_t)np;
                        j++;
                    }
                }
            } else {
                const int np = (int)C + (int)nb[p];
                B.rect[np] = A.rect[p];
                B.cnt[np] = A.cnt[p];
                B.xr[np] = -1;
                for (int u = 0; u < 4; u++) B.ch[4 * np + u] = 0;
            }
        }
        for (int k = 0; k < n; k++) {   // remap
            const int p = kn[k] & 0xFFFF;
            if (A.xr[p] >= 0) {
                const int q = kn[k] >> 16;
                int j = 0;
                for (int u = 0; u < q; u++) j += A.ch[4 * p + u] > 0;
                kn[k] = (uint32_t)((int)C - 1 - ((int)(nb[p] & 0xFFFF) + j));
            } else {
                kn[k] = C + nb[p];
            }
        }
        S = Snew;
        m = (int)M;
        cur ^= 1;
        if (fin) break;
        final_phase = next_final;
    }
    // retain the best key per node (first max response in candidate order)
    std::vector<uint32_t> best(S, 0), wk(S, 0);
    for (int k = 0; k < n; k++) {
        const uint32_t v = ((key[k] >> 24) << 24) | (0xFFFFFFu - (uint32_t)k);
        uint32_t& b = best[kn[k] & 0xFFFF];
        b = v > b ? v : b;
    }
    for (int k = 0; k < n; k++) {
        const int p = kn[k] & 0xFFFF;
        if (best[p] == (((key[k] >> 24) << 24) | (0xFFFFFFu - (uint32_t)k))) wk[p] = key[k];
    }
    for (int p = 0; p < S && p < cap; p++) out[p] = wk[p];
    return S;
}
