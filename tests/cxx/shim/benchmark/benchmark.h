// Minimal google-benchmark-compatible shim (test infrastructure): enough of
// the API for the reference's benchmarks/SortNBenchmark.cpp to compile
// unchanged (its third_party/benchmark submodule is empty here).  Each
// registered benchmark runs `--benchmark_min_iters` (default 1) iterations,
// selected by --benchmark_filter=<regex> (searched, as google-benchmark does), and prints wall ms/iteration.
#pragma once
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <regex>
#include <string>
#include <vector>

namespace benchmark {
enum TimeUnit { kNanosecond, kMicrosecond, kMillisecond, kSecond };

class State {
  public:
    explicit State(int iters, long long arg = 0) : left_(iters), total_(iters), arg_(arg) {}
    struct Iter {
        State* s;
        bool operator!=(const Iter&) const { return s->left_ > 0; }
        void operator++() { --s->left_; }
        int operator*() const { return 0; }
    };
    Iter begin() { return Iter{this}; }
    Iter end() { return Iter{this}; }
    std::map<std::string, double> counters;
    int iterations() const { return total_; }
    long long range(int) const { return arg_; }

  private:
    int left_, total_;
    long long arg_;
};

template <class T>
inline void DoNotOptimize(T const& v) {
    asm volatile("" : : "g"(&v) : "memory");
}
inline void ClobberMemory() { asm volatile("" : : : "memory"); }

namespace internal {
struct Bench {
    std::string name;
    std::function<void(State&)> fn;
    Bench* Unit(TimeUnit) { return this; }
    Bench* UseRealTime() { return this; }
    Bench* Iterations(int) { return this; }
    Bench* Arg(long long a) {
        args.push_back(a);
        return this;
    }
    Bench* DenseRange(long long lo, long long hi, long long step = 1) {
        for (long long a = lo; a <= hi; a += step) args.push_back(a);
        return this;
    }
    std::vector<long long> args;  // empty: one run without an argument
};
inline std::vector<Bench*>& all() {
    static std::vector<Bench*> v;
    return v;
}
inline Bench* add(const char* name, std::function<void(State&)> fn) {
    auto* b = new Bench{name, std::move(fn)};
    all().push_back(b);
    return b;
}
inline int run(int argc, char** argv) {
    std::string filter;
    int iters = 1;
    bool list = false;
    for (int i = 1; i < argc; ++i) {
        if (!std::strncmp(argv[i], "--benchmark_filter=", 19)) filter = argv[i] + 19;
        if (!std::strncmp(argv[i], "--benchmark_min_iters=", 22)) iters = std::atoi(argv[i] + 22);
        if (!std::strcmp(argv[i], "--benchmark_list_tests")) list = true;
    }
    for (auto* b : all()) {
        std::vector<std::pair<std::string, long long>> runs;
        if (b->args.empty()) runs.emplace_back(b->name, 0);
        for (long long a : b->args) runs.emplace_back(b->name + "/" + std::to_string(a), a);
        for (auto& r : runs) {
            if (!filter.empty() && !std::regex_search(r.first, std::regex(filter))) continue;
            if (list) {
                std::printf("%s\n", r.first.c_str());
                continue;
            }
            State st(iters, r.second);
            auto t0 = std::chrono::steady_clock::now();
            b->fn(st);
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            std::printf("%-28s %12.3f ms/iter  (%d iterations)", r.first.c_str(), ms / iters, iters);
            for (auto& kv : st.counters) std::printf("  %s=%g", kv.first.c_str(), kv.second);
            std::printf("\n");
            std::fflush(stdout);
        }
    }
    return 0;
}
}  // namespace internal
}  // namespace benchmark

#define BENCH_SHIM_CAT_(a, b) a##b
#define BENCH_SHIM_CAT(a, b) BENCH_SHIM_CAT_(a, b)
#define BENCHMARK(...) \
    static ::benchmark::internal::Bench* BENCH_SHIM_CAT(bench_shim_, __COUNTER__) = \
        ::benchmark::internal::add(#__VA_ARGS__, __VA_ARGS__)
#define BENCHMARK_MAIN() \
    int main(int argc, char** argv) { return ::benchmark::internal::run(argc, argv); } \
    int bench_shim_main_unused_
