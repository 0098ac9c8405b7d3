// Sampling profiler of the host code of one call (diagnostics only):
// GK_HOST_PROF=<microseconds> arms ITIMER_PROF for the scope of a HostProf
// object; every SIGPROF records the interrupted program counter as an offset
// into this library, and the destructor prints the most frequent offsets to
// stderr ("[gk hostprof] <samples> 0x<offset>"), to be symbolised against the
// same build with llvm-symbolizer --obj=glpk.js_amd/libglpk_mi355x.so.
// Samples outside the library are counted as "other".
#pragma once
#include <dlfcn.h>
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <unordered_map>
#include <vector>

namespace gk {

struct HostProf {
    static constexpr int CAP = 1 << 20;
    static inline std::atomic<int> n{0};
    static inline unsigned long long pcs[CAP];
    struct sigaction old {};
    bool on = false;
    static void handler(int, siginfo_t *, void *uc)
    {
        const int i = n.fetch_add(1, std::memory_order_relaxed);
        if (i < CAP) pcs[i] = (unsigned long long)((ucontext_t *)uc)->uc_mcontext.gregs[REG_RIP];
    }
    HostProf()
    {
        const char *e = std::getenv("GK_HOST_PROF");
        const int us = e ? std::atoi(e) : 0;
        if (us <= 0) return;
        n.store(0);
        struct sigaction sa {};
        sa.sa_sigaction = handler;
        sa.sa_flags = SA_SIGINFO | SA_RESTART;
        sigemptyset(&sa.sa_mask);
        if (sigaction(SIGPROF, &sa, &old) != 0) return;
        itimerval tv{{0, us}, {0, us}};
        on = setitimer(ITIMER_PROF, &tv, nullptr) == 0;
    }
    ~HostProf()
    {
        if (!on) return;
        itimerval tv{};
        (void)setitimer(ITIMER_PROF, &tv, nullptr);
        (void)sigaction(SIGPROF, &old, nullptr);
        Dl_info me{};
        (void)dladdr((void *)&handler, &me);
        const unsigned long long base = (unsigned long long)me.dli_fbase;
        std::unordered_map<unsigned long long, int> h;
        int other = 0;
        const int cnt = std::min(n.load(), CAP);
        for (int i = 0; i < cnt; i++) {
            Dl_info di{};
            if (dladdr((void *)pcs[i], &di) && di.dli_fbase == me.dli_fbase) h[pcs[i] - base]++;
            else other++;
        }
        std::vector<std::pair<int, unsigned long long>> v;
        for (auto &kv : h) v.emplace_back(kv.second, kv.first);
        std::sort(v.rbegin(), v.rend());
        fprintf(stderr, "[gk hostprof] %d samples, %d outside the library\n", cnt, other);
        for (size_t i = 0; i < v.size() && i < 60; i++) fprintf(stderr, "[gk hostprof] %d 0x%llx\n", v[i].first, v[i].second);
    }
};

}  // namespace gk
