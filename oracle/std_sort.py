"""TEST INFRASTRUCTURE (oracle) -- not part of the product path.

Restatement of the sort the reference's non_max_suppression runs: `torch.sort(scores,
descending=True)` (src/models/yolo_head.py:700) on the CPU is libstdc++'s std::sort (introsort)
over (value, index) pairs with comp(a, b) = a.value > b.value (torch's KeyValueCompDesc without
NaNs).  It is NOT stable: tied scores come out in whatever order introsort leaves them, and that
order decides which of two tied boxes NMS keeps first.  `tests/test_oracle_golden.py` pins this
restatement against torch.sort itself (heavy-tie inputs); the GPU kernel (hv_sort_desc_exact /
the tie path of hv_nms, csrc/hv_nms.hip) is held to it, including the heap-sort fallback reached
by forcing the depth limit.

The structure follows libstdc++ <bits/stl_algo.h> / <bits/stl_heap.h>: __introsort_loop
(_S_threshold = 16, depth limit 2*floor(log2 n)), __unguarded_partition_pivot with
__move_median_to_first(first, first+1, mid, last-1), __unguarded_partition, __partial_sort
(make_heap + sort_heap via __adjust_heap / __push_heap), __final_insertion_sort.
"""
from typing import List, Optional, Sequence


def std_sort_desc(vals: Sequence[float], depth_limit: Optional[int] = None) -> List[int]:
    """Indices of `vals` in the order std::sort(descending comparator) leaves them -- equal to
    torch.sort(torch.tensor(vals), descending=True).indices on the CPU.  depth_limit overrides
    std::sort's own 2*floor(log2 n) (None = the library's)."""
    a = [(float(v), i) for i, v in enumerate(vals)]

    def comp(x, y):
        return x[0] > y[0]

    def swap(i, j):
        a[i], a[j] = a[j], a[i]

    def median_to_first(res, x, y, z):
        if comp(a[x], a[y]):
            if comp(a[y], a[z]):
                swap(res, y)
            elif comp(a[x], a[z]):
                swap(res, z)
            else:
                swap(res, x)
        elif comp(a[x], a[z]):
            swap(res, x)
        elif comp(a[y], a[z]):
            swap(res, z)
        else:
            swap(res, y)

    def unguarded_partition(f, l, p):
        while True:
            while comp(a[f], a[p]):
                f += 1
            l -= 1
            while comp(a[p], a[l]):
                l -= 1
            if not f < l:
                return f
            swap(f, l)
            f += 1

    def adjust_heap(first, hole, length, value):
        top = hole
        child = hole
        while child < (length - 1) // 2:
            child = 2 * (child + 1)
            if comp(a[first + child], a[first + child - 1]):
                child -= 1
            a[first + hole] = a[first + child]
            hole = child
        if (length & 1) == 0 and child == (length - 2) // 2:
            child = 2 * (child + 1)
            a[first + hole] = a[first + child - 1]
            hole = child - 1
        parent = (hole - 1) // 2
        while hole > top and comp(a[first + parent], value):
            a[first + hole] = a[first + parent]
            hole = parent
            parent = (hole - 1) // 2
        a[first + hole] = value

    def heap_sort(f, l):
        n = l - f
        if n >= 2:
            parent = (n - 2) // 2
            while True:
                adjust_heap(f, parent, n, a[f + parent])
                if parent == 0:
                    break
                parent -= 1
        while l - f > 1:
            l -= 1
            v = a[l]
            a[l] = a[f]
            adjust_heap(f, 0, l - f, v)

    def introsort_loop(f, l, d):
        while l - f > 16:
            if d == 0:
                heap_sort(f, l)
                return
            d -= 1
            median_to_first(f, f + 1, f + (l - f) // 2, l - 1)
            cut = unguarded_partition(f + 1, l, f)
            introsort_loop(cut, l, d)
            l = cut

    n = len(a)
    if n:
        introsort_loop(0, n, 2 * (n.bit_length() - 1) if depth_limit is None else depth_limit)
        for i in range(1, n):                 # __final_insertion_sort (stable insertion)
            v = a[i]
            j = i
            while j > 0 and comp(v, a[j - 1]):
                a[j] = a[j - 1]
                j -= 1
            a[j] = v
    return [i for _, i in a]
