"""The order-exact parallel restatement of the reference's in-place partition (CPU).

Mesh::buildBVHMesh partitions a node's triangles with a single forward scan (Mesh.cuh:182-198):

    mid = start
    for i in start..end:  if centroid(i)[axis] < pos:  swap(tri[mid], tri[i]); mid += 1

Every other step of the reference builder is order-independent (min/max, counts, boxes), so this scan
is what decides the leaf order of the triangles, i.e. the index buffer and the hit tie-breaking.  The
GPU builder computes its result in parallel (csrc/crt_bvh_build.hip):

* the "less" triangles keep their relative order: the k-th one lands at start + k;
* the ">=" triangles form a queue in [mid, i]: a new ">=" triangle joins at the back; a "less" triangle
  at position i moves the queue's front to position i.  So every position j >= first ">=" is written
  exactly once more, by event j: with a ">=" triangle (its own) or, for a "less" triangle, with the
  element that position j - m_j holds, m_j = number of ">=" triangles before j (the queue length).
  The final content of the right block position j is therefore a[root(j)], where root follows
  j -> j - m_j through "less" positions until it reaches a ">=" position (pointer jumping: log2(n)
  parallel rounds).

This test checks that restatement against the sequential scan on adversarial flag patterns.
"""
import numpy as np
import pytest


def lomuto(flags):
    a = np.arange(len(flags))
    f = np.asarray(flags, bool)
    mid = 0
    for i in range(len(a)):
        if f[a[i]]:
            a[mid], a[i] = a[i], a[mid]
            mid += 1
    return a


def parallel(flags):
    f = np.asarray(flags, bool)
    n = len(f)
    less_before = np.concatenate([[0], np.cumsum(f)[:-1]]) if n else np.zeros(0, int)
    ge_before = np.arange(n) - less_before
    l_total = int(f.sum())
    out = np.empty(n, int)
    out[less_before[f]] = np.nonzero(f)[0]                     # stable left block
    ptr = np.where(f, np.arange(n) - ge_before, np.arange(n))   # "less": j -> j - m_j ; ">=": itself
    ptr = np.where(f & (ge_before == 0), np.arange(n), ptr)     # before the first ">=": never referenced
    rounds = 0
    while True:                                                # pointer jumping
        nxt = ptr[ptr]
        rounds += 1
        if np.array_equal(nxt, ptr):
            break
        ptr = nxt
    assert rounds <= max(1, int(np.ceil(np.log2(max(n, 2))))) + 1
    out[l_total:] = ptr[l_total:]
    return out


def cases():
    rng = np.random.default_rng(3)
    yield [True] * 17
    yield [False] * 17
    yield [False] + [True] * 40                                 # longest chains: queue of one
    yield [True] * 5 + [False] * 3 + [True] * 30
    yield [False, True] * 20
    yield [True, False] * 20
    yield [False] * 3 + [True] * 50 + [False] * 2
    for n in (1, 2, 3, 10, 33, 100, 1000, 4097):
        for p in (0.05, 0.5, 0.95):
            yield list(rng.random(n) < p)
    for _ in range(20):                                          # runs, like spatially coherent meshes
        n = int(rng.integers(30, 3000))
        runs = np.repeat(rng.random(n // 10 + 1) < 0.5, 10)[:n]
        yield list(runs)


@pytest.mark.parametrize("flags", list(cases()))
def test_parallel_partition_matches_reference_scan(flags):
    assert parallel(flags).tolist() == lomuto(flags).tolist()
