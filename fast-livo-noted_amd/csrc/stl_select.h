// stl_select.h — libstdc++'s std::nth_element, restated element for element
// for one GPU thread (and the host, for its test).
//
// The iVox k-NN (include/ivox3d/ivox3d.h:132-204, ivox3d_node.hpp:141-205)
// selects with std::nth_element and returns the survivors in the order the
// algorithm leaves them, which is not sorted; esti_plane (common_lib.h:670-702)
// then fits the 5 points in that row order.  To reproduce the reference's
// plane fit bit for bit, the device must leave the candidates in exactly the
// order libstdc++ does.  This is libstdc++'s introselect (bits/stl_algo.h:
// __introselect, __unguarded_partition_pivot, __move_median_to_first,
// __unguarded_partition, __insertion_sort, __heap_select; bits/stl_heap.h:
// __make_heap, __adjust_heap, __push_heap, __pop_heap), unchanged since GCC 4.x,
// over elements compared by their float key only (DistPoint::operator<,
// ivox3d_node.hpp:117: the double distance is a widened float, so comparing
// the floats orders them identically).
//
// `P` is anything indexable as a[i] -> SelElem& (a private array on the GPU,
// a global-memory slice in the overflow pass, a std::vector on the host).
#pragma once
#include <stdint.h>

#if defined(__HIP__)  // compiling HIP source (device + host)
#include <hip/hip_runtime.h>
#define SEL_HD __host__ __device__ __forceinline__
#else
#define SEL_HD inline
#endif

namespace livo {

struct SelElem {
    float d;      // squared distance (the DistPoint::dist, as float)
    uint32_t id;  // payload (map point position)
};

template <class P>
SEL_HD void sel_swap(P& a, int i, int j) {
    const SelElem t = a[i];
    a[i] = a[j];
    a[j] = t;
}

template <class P>
SEL_HD void sel_move_median_to_first(P& a, int result, int x, int y, int z) {
    if (a[x].d < a[y].d) {
        if (a[y].d < a[z].d)
            sel_swap(a, result, y);
        else if (a[x].d < a[z].d)
            sel_swap(a, result, z);
        else
            sel_swap(a, result, x);
    } else if (a[x].d < a[z].d) {
        sel_swap(a, result, x);
    } else if (a[y].d < a[z].d) {
        sel_swap(a, result, z);
    } else {
        sel_swap(a, result, y);
    }
}

template <class P>
SEL_HD int sel_unguarded_partition(P& a, int first, int last, int pivot) {
    const float pv = a[pivot].d;  // the pivot element is not moved by the partition
    while (true) {
        while (a[first].d < pv) ++first;
        --last;
        while (pv < a[last].d) --last;
        if (!(first < last)) return first;
        sel_swap(a, first, last);
        ++first;
    }
}

template <class P>
SEL_HD void sel_insertion_sort(P& a, int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
        const SelElem val = a[i];
        if (val.d < a[first].d) {
            for (int k = i; k > first; --k) a[k] = a[k - 1];  // move_backward
            a[first] = val;
        } else {  // __unguarded_linear_insert
            int hole = i, next = i - 1;
            while (val.d < a[next].d) {
                a[hole] = a[next];
                hole = next;
                --next;
            }
            a[hole] = val;
        }
    }
}

template <class P>
SEL_HD void sel_push_heap(P& a, int first, int hole, int top, SelElem value) {
    int parent = (hole - 1) / 2;
    while (hole > top && a[first + parent].d < value.d) {
        a[first + hole] = a[first + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a[first + hole] = value;
}

template <class P>
SEL_HD void sel_adjust_heap(P& a, int first, int hole, int len, SelElem value) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (a[first + second].d < a[first + second - 1].d) second--;
        a[first + hole] = a[first + second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        a[first + hole] = a[first + second - 1];
        hole = second - 1;
    }
    sel_push_heap(a, first, hole, top, value);
}

// std::__heap_select(first, middle, last): only reached when the introselect
// depth limit (2 floor(log2 n)) runs out.
template <class P>
SEL_HD void sel_heap_select(P& a, int first, int middle, int last) {
    const int len = middle - first;
    if (len >= 2) {  // __make_heap
        int parent = (len - 2) / 2;
        while (true) {
            sel_adjust_heap(a, first, parent, len, a[first + parent]);
            if (parent == 0) break;
            parent--;
        }
    }
    for (int i = middle; i < last; ++i)
        if (a[i].d < a[first].d) {  // __pop_heap(first, middle, i)
            const SelElem v = a[i];
            a[i] = a[first];
            sel_adjust_heap(a, first, 0, len, v);
        }
}

SEL_HD int sel_lg(int n) {  // std::__lg: floor(log2 n), n > 0
    int r = 0;
    while (n > 1) {
        n >>= 1;
        r++;
    }
    return r;
}

// std::nth_element(a + first, a + nth, a + last) with operator<.
template <class P>
SEL_HD void sel_nth_element(P& a, int first, int nth, int last) {
    if (first == last || nth == last) return;
    int depth = 2 * sel_lg(last - first);
    while (last - first > 3) {
        if (depth == 0) {
            sel_heap_select(a, first, nth + 1, last);
            sel_swap(a, first, nth);
            return;
        }
        --depth;
        // __unguarded_partition_pivot
        const int mid = first + (last - first) / 2;
        sel_move_median_to_first(a, first, first + 1, mid, last - 1);
        const int cut = sel_unguarded_partition(a, first + 1, last, first);
        if (cut <= nth)
            first = cut;
        else
            last = cut;
    }
    sel_insertion_sort(a, first, last);
}

}  // namespace livo
