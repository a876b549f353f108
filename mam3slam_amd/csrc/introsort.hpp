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

}  // namespace mam
