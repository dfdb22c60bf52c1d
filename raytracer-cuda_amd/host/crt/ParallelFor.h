// ParallelFor.h — the scene set-up's data-parallel host loops ("Scene creation").
#pragma once
#include <algorithm>
#include <cstddef>
#include <exception>
#include <thread>
#include <vector>

namespace CRT {

// f(r, b, e) handles range r, the contiguous indices [b, e) of [0, n), on up to 16 threads (the GPU box's CPU quota)
// of at least min_per_thread indices each.  Ranges are numbered in index order, so a caller that folds per range and
// then over the ranges in order gets the sequential fold.  Returns the number of ranges.
template <class F>
size_t parallel_ranges_indexed(size_t n, F&& f, size_t min_per_thread = (size_t)1 << 15) {
    const unsigned hw = std::thread::hardware_concurrency();
    const size_t T = std::max<size_t>(1, std::min<size_t>(std::min<size_t>(16, hw ? hw : 1),
                                                          (n + min_per_thread - 1) / min_per_thread));
    if (T == 1) {
        f((size_t)0, (size_t)0, n);
        return 1;
    }
    // an exception in a worker (std::bad_alloc) is rethrown here after every worker has joined, as the sequential loop
    // would have thrown it, instead of terminating the process
    std::vector<std::exception_ptr> err(T);
    auto run = [&f, &err, n, T](size_t t) {
        try {
            f(t, n * t / T, n * (t + 1) / T);
        } catch (...) {
            err[t] = std::current_exception();
        }
    };
    std::vector<std::thread> th;
    th.reserve(T - 1);
    size_t started = 1;   // ranges 1 .. started-1 have a thread
    try {
        for (; started < T; ++started) th.emplace_back(run, started);
    } catch (...) {
        // no thread could be started (std::system_error): the ranges without one run on this thread, after the
        // others, so no started thread is left unjoined
    }
    run(0);
    for (size_t t = started; t < T; ++t) run(t);
    for (auto& x : th) x.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
    return T;
}

// f(b, e) for each range of parallel_ranges_indexed.
template <class F>
void parallel_ranges(size_t n, F&& f, size_t min_per_thread = (size_t)1 << 15) {
    parallel_ranges_indexed(n, [&f](size_t, size_t b, size_t e) { f(b, e); }, min_per_thread);
}

}  // namespace CRT
