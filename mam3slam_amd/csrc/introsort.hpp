// introsort.hpp — exact emulation of libstdc++'s std::sort (GCC 11 bits/stl_algo.h, stl_heap.h) on
// (key, payload) pairs compared by key only.
//
// Why: DistributeOctTree (reference src/ORBextractor.cc:689) sorts (node size, node*) pairs with
// compareNodes (:538-553), a non-total order — nodes of equal size and equal UL.x tie, and std::sort is
// unstable, so the order ties come out in is whatever libstdc++'s introsort produces. Because the
// expansion order decides the final keypoint order, a bit-exact device implementation must replay the
// same algorithm: median-of-3 pivot to *first, unguarded Hoare partition, recursion on the right part,
// heapsort once the 2*floor(log2 n) depth budget is spent, final insertion sort with threshold 16.
//
// Usable from host and device (tests compile it with g++ against the real std::sort).
#pragma once

#include <stdint.h>

#if !defined(__HIPCC__)
#include <algorithm>
#include <vector>
#endif

#if defined(__HIPCC__)
#define MAM_HD __host__ __device__ __forceinline__
#else
#define MAM_HD inline
#endif

namespace mam {

// Sort element: 32-bit key (compared) + 32-bit payload (carried). Pointer-based like the STL.
struct SortEl {
    uint32_t key;
    uint32_t val;
};

MAM_HD bool sl_less(const SortEl& a, const SortEl& b) { return a.key < b.key; }

MAM_HD void sl_swap(SortEl* a, SortEl* b) {
    SortEl t = *a;
    *a = *b;
    *b = t;
}

MAM_HD int sl_lg(int n) {  // std::__lg: floor(log2 n) for n > 0
    int r = 0;
    while (n > 1) { n >>= 1; ++r; }
    return r;
}

// std::__push_heap
MAM_HD void sl_push_heap(SortEl* first, int holeIndex, int topIndex, SortEl value) {
    int parent = (holeIndex - 1) / 2;
    while (holeIndex > topIndex && sl_less(first[parent], value)) {
        first[holeIndex] = first[parent];
        holeIndex = parent;
        parent = (holeIndex - 1) / 2;
    }
    first[holeIndex] = value;
}

// std::__adjust_heap
MAM_HD void sl_adjust_heap(SortEl* first, int holeIndex, int len, SortEl value) {
    const int topIndex = holeIndex;
    int secondChild = holeIndex;
    while (secondChild < (len - 1) / 2) {
        secondChild = 2 * (secondChild + 1);
        if (sl_less(first[secondChild], first[secondChild - 1])) secondChild--;
        first[holeIndex] = first[secondChild];
        holeIndex = secondChild;
    }
    if ((len & 1) == 0 && secondChild == (len - 2) / 2) {
        secondChild = 2 * (secondChild + 1);
        first[holeIndex] = first[secondChild - 1];
        holeIndex = secondChild - 1;
    }
    sl_push_heap(first, holeIndex, topIndex, value);
}

// std::__make_heap
MAM_HD void sl_make_heap(SortEl* first, SortEl* last) {
    const int len = (int)(last - first);
    if (len < 2) return;
    int parent = (len - 2) / 2;
    while (true) {
        SortEl value = first[parent];
        sl_adjust_heap(first, parent, len, value);
        if (parent == 0) return;
        parent--;
    }
}

// std::__pop_heap(first, last, result)
MAM_HD void sl_pop_heap(SortEl* first, SortEl* last, SortEl* result) {
    SortEl value = *result;
    *result = *first;
    sl_adjust_heap(first, 0, (int)(last - first), value);
}

// std::__partial_sort(first, middle, last) with middle == last: __heap_select + __sort_heap
MAM_HD void sl_heap_sort(SortEl* first, SortEl* last) {
    sl_make_heap(first, last);  // __heap_select(first, last, last): no element beyond middle
    while (last - first > 1) {
        --last;
        sl_pop_heap(first, last, last);
    }
}

// std::__move_median_to_first
MAM_HD void sl_move_median_to_first(SortEl* result, SortEl* a, SortEl* b, SortEl* c) {
    if (sl_less(*a, *b)) {
        if (sl_less(*b, *c)) sl_swap(result, b);
        else if (sl_less(*a, *c)) sl_swap(result, c);
        else sl_swap(result, a);
    } else if (sl_less(*a, *c)) sl_swap(result, a);
    else if (sl_less(*b, *c)) sl_swap(result, c);
    else sl_swap(result, b);
}

// std::__unguarded_partition
MAM_HD SortEl* sl_unguarded_partition(SortEl* first, SortEl* last, SortEl* pivot) {
    while (true) {
        while (sl_less(*first, *pivot)) ++first;
        --last;
        while (sl_less(*pivot, *last)) --last;
        if (!(first < last)) return first;
        sl_swap(first, last);
        ++first;
    }
}

// std::__unguarded_partition_pivot
MAM_HD SortEl* sl_partition_pivot(SortEl* first, SortEl* last) {
    SortEl* mid = first + (last - first) / 2;
    sl_move_median_to_first(first, first + 1, mid, last - 1);
    return sl_unguarded_partition(first + 1, last, first);
}

// std::__unguarded_linear_insert
MAM_HD void sl_unguarded_linear_insert(SortEl* last) {
    SortEl val = *last;
    SortEl* next = last - 1;
    while (sl_less(val, *next)) {
        *last = *next;
        last = next;
        --next;
    }
    *last = val;
}

// std::__insertion_sort
MAM_HD void sl_insertion_sort(SortEl* first, SortEl* last) {
    if (first == last) return;
    for (SortEl* i = first + 1; i != last; ++i) {
        if (sl_less(*i, *first)) {
            SortEl val = *i;
            for (SortEl* p = i; p != first; --p) *p = *(p - 1);  // move_backward(first, i, i + 1)
            *first = val;
        } else {
            sl_unguarded_linear_insert(i);
        }
    }
}

// std::__final_insertion_sort
MAM_HD void sl_final_insertion_sort(SortEl* first, SortEl* last) {
    if (last - first > 16) {
        sl_insertion_sort(first, first + 16);
        for (SortEl* i = first + 16; i != last; ++i) sl_unguarded_linear_insert(i);
    } else {
        sl_insertion_sort(first, last);
    }
}

// std::__introsort_loop with the recursion on [cut, last) replaced by an explicit stack. The ranges are
// disjoint and each carries its own depth budget, so the processing order does not change the result.
MAM_HD void sl_introsort_loop(SortEl* first, SortEl* last, int depth_limit) {
    SortEl* stk_first[64];
    SortEl* stk_last[64];
    int stk_depth[64];
    int sp = 0;
    stk_first[sp] = first; stk_last[sp] = last; stk_depth[sp] = depth_limit; ++sp;
    while (sp > 0) {
        --sp;
        SortEl* f = stk_first[sp];
        SortEl* l = stk_last[sp];
        int d = stk_depth[sp];
        while (l - f > 16) {
            if (d == 0) {
                sl_heap_sort(f, l);
                break;
            }
            --d;
            SortEl* cut = sl_partition_pivot(f, l);
            stk_first[sp] = cut; stk_last[sp] = l; stk_depth[sp] = d; ++sp;  // __introsort_loop(cut, last, d)
            l = cut;
        }
    }
}

// std::sort(first, last, comp)
MAM_HD void stl_sort(SortEl* first, SortEl* last) {
    if (first != last) {
        sl_introsort_loop(first, last, sl_lg((int)(last - first)) * 2);
        sl_final_insertion_sort(first, last);
    }
}

// ---------------------------------------------------------------------------------------------------------
// Data-parallel formulation of the same algorithm (used by one wave on the device for n <= 64).
//
// __unguarded_partition(first+1, last, pivot at *first) as stoppers: L_k = k-th position from the left in
// [first+1, last) with !(a < pivot), R_k = k-th position from the right in [first, last) with !(pivot < a)
// (*first, the pivot itself, is the sentinel). Every swap exchanges L_k and R_k of the ORIGINAL values as long
// as L_k < R_k; with K the first k where L_k >= R_k, the returned cut is L_0 when K = 0, else
// min(L_K, R_{K-1}) (after swap K-1 the left scan meets the swapped value at R_{K-1}, which stops it).
// Ranges at most 16 long are left for the final insertion sort, which is stable, so it equals a stable sort
// of the post-partition array by key. These are exactly the operations the sequential code performs.
MAM_HD int sl_partition_model(SortEl* a, int first, int last) {
    const int mid = first + (last - first) / 2;
    sl_move_median_to_first(a + first, a + first + 1, a + mid, a + last - 1);
    const SortEl pv = a[first];
    int Lp[1024], Rp[1024];
    int nl = 0, nr = 0;
    for (int p = first + 1; p < last; p++)
        if (!sl_less(a[p], pv)) Lp[nl++] = p;
    for (int p = last - 1; p >= first; p--)
        if (!sl_less(pv, a[p])) Rp[nr++] = p;
    int K = 0;
    while (K < nl && K < nr && Lp[K] < Rp[K]) K++;
    for (int k = 0; k < K; k++) sl_swap(a + Lp[k], a + Rp[k]);
    if (K == 0) return Lp[0];
    return K < nl ? (Lp[K] < Rp[K - 1] ? Lp[K] : Rp[K - 1]) : Rp[K - 1];
}

// Host model of the whole data-parallel sort (n <= 1024): same result as stl_sort.
inline void stl_sort_model(SortEl* a, int n) {
    if (n == 0) return;
    int sf[64], sl[64], sd[64], sp = 0;
    sf[sp] = 0; sl[sp] = n; sd[sp] = sl_lg(n) * 2; ++sp;
    while (sp > 0) {
        --sp;
        int f = sf[sp], l = sl[sp], d = sd[sp];
        while (l - f > 16) {
            if (d == 0) { sl_heap_sort(a + f, a + l); break; }
            --d;
            const int cut = sl_partition_model(a, f, l);
            sf[sp] = cut; sl[sp] = l; sd[sp] = d; ++sp;
            l = cut;
        }
    }
    // final insertion sort == stable sort by key
    SortEl tmp[1024];
    for (int i = 0; i < n; i++) {
        int r = 0;
        for (int q = 0; q < n; q++) r += sl_less(a[q], a[i]) || (a[q].key == a[i].key && q < i);
        tmp[r] = a[i];
    }
    for (int i = 0; i < n; i++) a[i] = tmp[i];
}

// The same with the final insertion sort restated per leaf: the partitions leave [0, n) tiled by leaves (ranges of at
// most 16 elements, or heap-sorted ranges), and every key of a leaf is <= every key of a later leaf (a partition puts
// keys <= pivot left of the cut and keys >= pivot right of it). A stable sort of the whole array therefore equals the
// leaves stable-sorted one by one in place: an element's final position is its leaf's start + its stable rank inside
// the leaf (the device's final stage: at most 16 comparisons per element instead of n).
#if !defined(__HIPCC__)
inline void stl_sort_model_leaf(SortEl* a, int n) {
    if (n == 0) return;
    int sf[64], sl[64], sd[64], sp = 0;
    std::vector<int> leaf_start;
    sf[sp] = 0; sl[sp] = n; sd[sp] = sl_lg(n) * 2; ++sp;
    while (sp > 0) {
        --sp;
        int f = sf[sp], l = sl[sp], d = sd[sp];
        while (l - f > 16) {
            if (d == 0) { sl_heap_sort(a + f, a + l); break; }
            --d;
            const int cut = sl_partition_model(a, f, l);
            sf[sp] = cut; sl[sp] = l; sd[sp] = d; ++sp;
            l = cut;
        }
        if (f < l) leaf_start.push_back(f);
    }
    std::sort(leaf_start.begin(), leaf_start.end());
    std::vector<SortEl> tmp(a, a + n);
    for (size_t j = 0; j < leaf_start.size(); j++) {
        const int s0 = leaf_start[j], s1 = j + 1 < leaf_start.size() ? leaf_start[j + 1] : n;
        for (int p = s0; p < s1; p++) {
            int r = 0;
            for (int q = s0; q < s1; q++) r += sl_less(tmp[q], tmp[p]) || (tmp[q].key == tmp[p].key && q < p);
            a[s0 + r] = tmp[p];
        }
    }
}
#endif

#if defined(__HIPCC__)
// One full wave sorts arr[0, n) (n <= 64 * E, in LDS) exactly like stl_sort: E elements per lane in registers
// (position e * 64 + lane), the stoppers of each partition found by ballot and paired through LDS by rank. Ranges
// whose depth budget runs out fall back to lane 0's sequential heapsort on LDS (the same operations as stl_sort).
// scratch: LDS, >= MAM_SORT_WAVE_SCRATCH(E) ints, private to this wave.
#define MAM_SORT_WAVE_SCRATCH(E) (3 * 24 + 2 * 64 * (E))
template <int E>
__device__ __forceinline__ void stl_sort_wave(SortEl* arr, int n, int* scratch) {
    const int lane = threadIdx.x & 63;
    if (n <= 1) return;
    int* const stack = scratch;
    int* const Lpos = scratch + 72;
    int* const Rpos = scratch + 72 + 64 * E;
    uint32_t key[E], val[E];
#pragma unroll
    for (int e = 0; e < E; e++) {
        const int p = e * 64 + lane;
        key[e] = p < n ? arr[p].key : 0xFFFFFFFFu;
        val[e] = p < n ? arr[p].val : 0u;
    }
    auto get_key = [&](int p) -> uint32_t {
        uint32_t r = 0;
#pragma unroll
        for (int e = 0; e < E; e++) {
            const uint32_t v = __shfl(key[e], p & 63, 64);
            if ((p >> 6) == e) r = v;
        }
        return r;
    };
    auto get_val = [&](int p) -> uint32_t {
        uint32_t r = 0;
#pragma unroll
        for (int e = 0; e < E; e++) {
            const uint32_t v = __shfl(val[e], p & 63, 64);
            if ((p >> 6) == e) r = v;
        }
        return r;
    };
    // wave-uniform positions: v_readlane (scalar result), no LDS round trip
    auto key_at = [&](int p) -> uint32_t {
        uint32_t r = 0;
#pragma unroll
        for (int e = 0; e < E; e++)
            if ((p >> 6) == e) r = (uint32_t)__builtin_amdgcn_readlane((int)key[e], p & 63);
        return r;
    };
    auto val_at = [&](int p) -> uint32_t {
        uint32_t r = 0;
#pragma unroll
        for (int e = 0; e < E; e++)
            if ((p >> 6) == e) r = (uint32_t)__builtin_amdgcn_readlane((int)val[e], p & 63);
        return r;
    };
    const uint64_t below = (1ull << lane) - 1ull;
    const uint64_t above = ~(below | (1ull << lane));
    int sp = 0;
    int cf = 0, cl = n, cd = sl_lg(n) * 2;
    while (true) {
        while (cl - cf > 16) {
            if (cd == 0) {
#pragma unroll
                for (int e = 0; e < E; e++) {
                    const int p = e * 64 + lane;
                    if (p < n) { arr[p].key = key[e]; arr[p].val = val[e]; }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (lane == 0) sl_heap_sort(arr + cf, arr + cl);
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int e = 0; e < E; e++) {
                    const int p = e * 64 + lane;
                    if (p < n) { key[e] = arr[p].key; val[e] = arr[p].val; }
                }
                break;
            }
            --cd;
            // __move_median_to_first(first, first + 1, mid, last - 1)
            const int mid = cf + (cl - cf) / 2;
            const uint32_t ka = key_at(cf + 1), kb = key_at(mid), kc = key_at(cl - 1);
            int sw;
            if (ka < kb) sw = kb < kc ? mid : (ka < kc ? cl - 1 : cf + 1);
            else sw = ka < kc ? cf + 1 : (kb < kc ? cl - 1 : mid);
            {
                const uint32_t kf = key_at(cf), vf = val_at(cf), ks = key_at(sw), vs = val_at(sw);
#pragma unroll
                for (int e = 0; e < E; e++) {
                    const int p = e * 64 + lane;
                    if (p == cf) { key[e] = ks; val[e] = vs; }
                    else if (p == sw) { key[e] = kf; val[e] = vf; }
                }
            }
            const uint32_t pv = key_at(cf);
            uint64_t mL[E], mR[E];
            bool isL[E], isR[E];
            int nl = 0, nr = 0;
#pragma unroll
            for (int e = 0; e < E; e++) {
                const int p = e * 64 + lane;
                const bool inr = p > cf && p < cl;
                isL[e] = inr && !(key[e] < pv);                    // left scan stops here
                isR[e] = (inr && !(pv < key[e])) || p == cf;       // right scan stops here (pivot = sentinel)
                mL[e] = __ballot(isL[e]);
                mR[e] = __ballot(isR[e]);
                nl += __popcll(mL[e]);
                nr += __popcll(mR[e]);
            }
            int rankL[E], rankR[E];
            {
                int lo = 0;
#pragma unroll
                for (int e = 0; e < E; e++) {
                    rankL[e] = lo + __popcll(mL[e] & below);        // k-th from the left
                    lo += __popcll(mL[e]);
                }
                int hi = 0;
#pragma unroll
                for (int e = E - 1; e >= 0; e--) {
                    rankR[e] = hi + __popcll(mR[e] & above);        // k-th from the right
                    hi += __popcll(mR[e]);
                }
            }
#pragma unroll
            for (int e = 0; e < E; e++) {
                if (isL[e]) Lpos[rankL[e]] = e * 64 + lane;
                if (isR[e]) Rpos[rankR[e]] = e * 64 + lane;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            int src[E];
            int K = 0;
#pragma unroll
            for (int e = 0; e < E; e++) {
                const int partnerL = (isL[e] && rankL[e] < nr) ? Rpos[rankL[e]] : -1;
                const bool swapL = partnerL > e * 64 + lane;        // swap k happens iff L_k < R_k (monotone in k)
                src[e] = swapL ? partnerL : -1;
                K += __popcll(__ballot(swapL));
            }
#pragma unroll
            for (int e = 0; e < E; e++) {
                if (src[e] < 0) src[e] = (isR[e] && rankR[e] < K) ? Lpos[rankR[e]] : e * 64 + lane;
            }
            uint32_t nk[E], nv[E];
#pragma unroll
            for (int e = 0; e < E; e++) { nk[e] = get_key(src[e]); nv[e] = get_val(src[e]); }
#pragma unroll
            for (int e = 0; e < E; e++) { key[e] = nk[e]; val[e] = nv[e]; }
            // returned cut: L_0 if no swap, else min(L_K, R_{K-1}) (L_K absent -> R_{K-1})
            int cut;
            if (K == 0) cut = Lpos[0];
            else {
                const int rk = Rpos[K - 1];
                cut = (K < nl && Lpos[K] < rk) ? Lpos[K] : rk;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) { stack[3 * sp] = cut; stack[3 * sp + 1] = cl; stack[3 * sp + 2] = cd; }
            ++sp;
            cl = cut;
        }
        if (sp == 0) break;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        --sp;
        cf = stack[3 * sp];
        cl = stack[3 * sp + 1];
        cd = stack[3 * sp + 2];
    }
    // final insertion sort == stable sort by key of the partitioned array: rank by (key, position)
    int r[E];
#pragma unroll
    for (int e = 0; e < E; e++) r[e] = 0;
    for (int q = 0; q < n; q++) {
        const uint32_t kq = key_at(q);
#pragma unroll
        for (int e = 0; e < E; e++) r[e] += (kq < key[e]) || (kq == key[e] && q < e * 64 + lane);
    }
#pragma unroll
    for (int e = 0; e < E; e++) {
        if (e * 64 + lane < n) { arr[r[e]].key = key[e]; arr[r[e]].val = val[e]; }
    }
}

// stl_sort_wave's partitions with two LDS round trips each (both stopper pairings read at once, the elements moved by
// an LDS scatter to their destinations instead of per-slot shuffles, the cut found by ballots) and the final insertion
// sort per leaf (stl_sort_model_leaf): each element ranked against the at most 16 elements of its leaf. Same result.
// scratch: LDS, >= MAM_SORT_WAVE2_SCRATCH(E) ints, private to this wave.
#define MAM_SORT_WAVE2_SCRATCH(E) (3 * 24 + 4 * 64 * (E))
template <int E>
__device__ __forceinline__ void stl_sort_wave2(SortEl* arr, int n, int* scratch) {
    const int lane = threadIdx.x & 63;
    if (n <= 1) return;
    int* const stack = scratch;
    int* const Lpos = scratch + 72;
    int* const Rpos = Lpos + 64 * E;
    SortEl* const tmp = reinterpret_cast<SortEl*>(Rpos + 64 * E);
    uint32_t key[E], val[E];
#pragma unroll
    for (int e = 0; e < E; e++) {
        const int p = e * 64 + lane;
        key[e] = p < n ? arr[p].key : 0xFFFFFFFFu;
        val[e] = p < n ? arr[p].val : 0u;
    }
    auto key_at = [&](int p) -> uint32_t {   // wave-uniform position
        uint32_t r = 0;
#pragma unroll
        for (int e = 0; e < E; e++)
            if ((p >> 6) == e) r = (uint32_t)__builtin_amdgcn_readlane((int)key[e], p & 63);
        return r;
    };
    auto val_at = [&](int p) -> uint32_t {
        uint32_t r = 0;
#pragma unroll
        for (int e = 0; e < E; e++)
            if ((p >> 6) == e) r = (uint32_t)__builtin_amdgcn_readlane((int)val[e], p & 63);
        return r;
    };
    // position of the first set bit of a wave-uniform (64 E)-bit mask (-1 if none)
    auto first_bit = [&](const uint64_t* m) -> int {
        int r = -1;
#pragma unroll
        for (int e = E - 1; e >= 0; e--)
            if (m[e]) r = 64 * e + __ffsll((unsigned long long)m[e]) - 1;
        return r;
    };
    const uint64_t below = (1ull << lane) - 1ull;
    const uint64_t above = ~(below | (1ull << lane));
    uint64_t leaf[E];
#pragma unroll
    for (int e = 0; e < E; e++) leaf[e] = 0;
    int sp = 0;
    int cf = 0, cl = n, cd = sl_lg(n) * 2;
    while (true) {
        while (cl - cf > 16) {
            if (cd == 0) {   // depth budget spent: lane 0 heap-sorts the range in LDS (stl_sort's operations)
#pragma unroll
                for (int e = 0; e < E; e++) {
                    const int p = e * 64 + lane;
                    if (p < n) { arr[p].key = key[e]; arr[p].val = val[e]; }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                if (lane == 0) sl_heap_sort(arr + cf, arr + cl);
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int e = 0; e < E; e++) {
                    const int p = e * 64 + lane;
                    if (p < n) { key[e] = arr[p].key; val[e] = arr[p].val; }
                }
                break;
            }
            --cd;
            // __move_median_to_first(first, first + 1, mid, last - 1)
            const int mid = cf + (cl - cf) / 2;
            const uint32_t ka = key_at(cf + 1), kb = key_at(mid), kc = key_at(cl - 1);
            int sw;
            if (ka < kb) sw = kb < kc ? mid : (ka < kc ? cl - 1 : cf + 1);
            else sw = ka < kc ? cf + 1 : (kb < kc ? cl - 1 : mid);
            const uint32_t kf = key_at(cf), vf = val_at(cf), ks = key_at(sw), vs = val_at(sw);
#pragma unroll
            for (int e = 0; e < E; e++) {
                const int p = e * 64 + lane;
                if (p == cf) { key[e] = ks; val[e] = vs; }
                else if (p == sw) { key[e] = kf; val[e] = vf; }
            }
            const uint32_t pv = ks;
            uint64_t mL[E], mR[E];
            bool isL[E], isR[E];
            int nl = 0, nr = 0;
#pragma unroll
            for (int e = 0; e < E; e++) {
                const int p = e * 64 + lane;
                const bool inr = p > cf && p < cl;
                isL[e] = inr && !(key[e] < pv);                    // left scan stops here
                isR[e] = (inr && !(pv < key[e])) || p == cf;       // right scan stops here (pivot = sentinel)
                mL[e] = __ballot(isL[e]);
                mR[e] = __ballot(isR[e]);
                nl += __popcll(mL[e]);
                nr += __popcll(mR[e]);
            }
            int rankL[E], rankR[E];
            {
                int lo = 0;
#pragma unroll
                for (int e = 0; e < E; e++) {
                    rankL[e] = lo + __popcll(mL[e] & below);        // k-th from the left
                    lo += __popcll(mL[e]);
                }
                int hi = 0;
#pragma unroll
                for (int e = E - 1; e >= 0; e--) {
                    rankR[e] = hi + __popcll(mR[e] & above);        // k-th from the right
                    hi += __popcll(mR[e]);
                }
            }
#pragma unroll
            for (int e = 0; e < E; e++) {
                if (isL[e]) Lpos[rankL[e]] = e * 64 + lane;
                if (isR[e]) Rpos[rankR[e]] = e * 64 + lane;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            // both pairings read at once: L_k's partner R_k, R_k's partner L_k; swap k happens iff L_k < R_k (monotone
            // in k, so the swaps are k < K)
            int dst[E];
            int K = 0;
#pragma unroll
            for (int e = 0; e < E; e++) {
                const int p = e * 64 + lane;
                const int pl = (isL[e] && rankL[e] < nr) ? Rpos[rankL[e]] : -1;
                const int pr = (isR[e] && rankR[e] < nl) ? Lpos[rankR[e]] : -1;
                const bool swapL = pl > p;
                K += __popcll(__ballot(swapL));
                dst[e] = swapL ? pl : (pr >= 0 ? -2 - pr : p);   // R stoppers decided once K is known
            }
            uint64_t mK[E], mKR[E], mL0[E];
#pragma unroll
            for (int e = 0; e < E; e++) {
                if (dst[e] <= -2) dst[e] = rankR[e] < K ? -2 - dst[e] : e * 64 + lane;
                mK[e] = __ballot(isL[e] && rankL[e] == K);          // L_K
                mKR[e] = __ballot(isR[e] && rankR[e] == K - 1);     // R_{K-1}
                mL0[e] = mL[e];
            }
            // returned cut: L_0 if no swap, else min(L_K, R_{K-1}) (L_K absent -> R_{K-1})
            int cut;
            if (K == 0) cut = first_bit(mL0);
            else {
                const int rk = first_bit(mKR);
                const int lk = K < nl ? first_bit(mK) : -1;
                cut = (lk >= 0 && lk < rk) ? lk : rk;
            }
            // move every element to its destination through LDS
#pragma unroll
            for (int e = 0; e < E; e++) {
                const int p = e * 64 + lane;
                if (p < n) { tmp[dst[e]].key = key[e]; tmp[dst[e]].val = val[e]; }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int e = 0; e < E; e++) {
                const int p = e * 64 + lane;
                if (p < n) { key[e] = tmp[p].key; val[e] = tmp[p].val; }
            }
            if (lane == 0) { stack[3 * sp] = cut; stack[3 * sp + 1] = cl; stack[3 * sp + 2] = cd; }
            ++sp;
            cl = cut;
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        if (cf < cl) {   // [cf, cl) is a leaf
#pragma unroll
            for (int e = 0; e < E; e++)
                if ((cf >> 6) == e) leaf[e] |= 1ull << (cf & 63);
        }
        if (sp == 0) break;
        --sp;
        cf = stack[3 * sp];
        cl = stack[3 * sp + 1];
        cd = stack[3 * sp + 2];
    }
    // final insertion sort, per leaf: position = leaf start + stable rank inside the leaf
#pragma unroll
    for (int e = 0; e < E; e++) {
        const int p = e * 64 + lane;
        if (p < n) { tmp[p].key = key[e]; tmp[p].val = val[e]; }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    int dpos[E];
#pragma unroll
    for (int e = 0; e < E; e++) {
        const int p = e * 64 + lane;
        dpos[e] = -1;
        if (p < n) {
            int s0 = 0, s1 = n;   // leaf [s0, s1) holding p: last leaf start <= p, first leaf start > p
#pragma unroll
            for (int e2 = 0; e2 < E; e2++) {
                uint64_t m = leaf[e2];
                const int o = p - 64 * e2;
                if (o < 0) m = 0;
                else if (o < 63) m &= (2ull << o) - 1ull;
                if (m) s0 = 64 * e2 + 63 - __clzll((long long)m);
            }
#pragma unroll
            for (int e2 = E - 1; e2 >= 0; e2--) {
                uint64_t m = leaf[e2];
                const int o = p - 64 * e2;
                if (o >= 63) m = 0;
                else if (o >= 0) m &= ~((2ull << o) - 1ull);
                if (m) s1 = 64 * e2 + __ffsll((unsigned long long)m) - 1;
            }
            int r = 0;
            for (int q = s0; q < s1; q++) {
                const uint32_t kq = tmp[q].key;
                r += (kq < key[e]) || (kq == key[e] && q < p);
            }
            dpos[e] = s0 + r;
        }
    }
#pragma unroll
    for (int e = 0; e < E; e++)
        if (dpos[e] >= 0) { arr[dpos[e]].key = key[e]; arr[dpos[e]].val = val[e]; }
}
#endif

}  // namespace mam
