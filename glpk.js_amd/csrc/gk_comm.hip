// Collective for the sharded branch and bound, inside the
// library: one process per GPU, every rank holding a gk_comm.
//
// The only collective the B&B needs is an all-gather of a fixed-size byte
// block per sync epoch ({incumbent, best bound, open nodes, active} and the
// node descriptors handed from busy to idle ranks, gk_mip.hip shard_epoch),
// plus one at the end that agrees on the winning incumbent.  Two transports:
//   RCCL (ncclAllGather over xGMI) when every rank drives its own device —
//     the 8-GPU node; the unique id travels over the bootstrap connection;
//   TCP through rank 0 (127.0.0.1 / a host address) otherwise — ranks that
//     share a device (RCCL refuses duplicate GPUs), CPU-only tests.
// The bootstrap is always the TCP star: rank 0 listens on addr ("host:port"),
// the others connect and announce their rank.  RCCL is loaded with dlopen
// (RTLD_LOCAL): the process may already carry another RCCL build (torch's).
//
// Between the epochs, ranks on one host share the incumbent through one word
// of shared memory (an atomic min on an order-preserving image
// of the objective): every rank publishes its incumbent after each batch and
// prunes its next batch with the best of all, instead of waiting for the
// next all-gather.  Rank 0 creates the segment (POSIX shm, unlinked as soon
// as every rank has mapped it, so nothing outlives the processes); ranks on
// different hosts fall back to the epoch exchange alone.
#include "../../include/glpk_mi355x.h"
#include "gk_internal.h"
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <arpa/inet.h>
#include <dlfcn.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cfloat>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace gk {
void set_err(const char *fmt, ...);
}
int gk_ctx_device(gk_ctx *);
// gk_ios_driver_sharded with a live incumbent between the epochs (gk_mip.hip)
extern "C" int gk_ios_driver_sharded_inc(gk_ctx *ctx, gk_mip *mip, const gk_iocp *parm, const gk_ios_shard *shard,
                                         double (*inc)(void *info, double mine), void *inc_info);

namespace {

struct Rccl {
    void *lib = nullptr;
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init = nullptr;
    decltype(&ncclAllGather) allgather = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclCommAbort) abort = nullptr;   // optional
    bool load()
    {
        if (lib) return true;
        for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            lib = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (lib) break;
        }
        if (!lib) return false;
        get_id = (decltype(get_id))dlsym(lib, "ncclGetUniqueId");
        init = (decltype(init))dlsym(lib, "ncclCommInitRank");
        allgather = (decltype(allgather))dlsym(lib, "ncclAllGather");
        destroy = (decltype(destroy))dlsym(lib, "ncclCommDestroy");
        abort = (decltype(abort))dlsym(lib, "ncclCommAbort");
        return get_id && init && allgather && destroy;
    }
};

bool send_all(int fd, const void *p, size_t n)
{
    const char *c = (const char *)p;
    while (n) {
        const ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return false;
        c += k;
        n -= (size_t)k;
    }
    return true;
}

bool recv_all(int fd, void *p, size_t n)
{
    char *c = (char *)p;
    while (n) {
        const ssize_t k = ::recv(fd, c, n, 0);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return false;
        c += k;
        n -= (size_t)k;
    }
    return true;
}

// data links: no Nagle delay, and a receive timeout (GK_COMM_TIMEOUT_S,
// default 600 s) so that a rank whose peer died or left the collective
// sequence gets an error return instead of blocking forever
void nodelay(int fd)
{
    int one = 1;
    (void)setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    static const int tmo = [] {
        const char *e = std::getenv("GK_COMM_TIMEOUT_S");
        const int v = e ? std::atoi(e) : 600;
        return v > 0 ? v : 600;
    }();
    timeval tv{tmo, 0};
    (void)setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
}

// a double's order as an unsigned integer's (non-negative: the sign bit set;
// negative: all bits inverted), so that the minimum is one integer atomic
unsigned long long ord_key(double v)
{
    unsigned long long b;
    std::memcpy(&b, &v, sizeof b);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
double ord_val(unsigned long long k)
{
    const unsigned long long b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    double v;
    std::memcpy(&v, &b, sizeof v);
    return v;
}

}  // namespace

struct gk_comm {
    int rank = 0, size = 1, backend = GK_COMM_TCP;
    int ramp_nodes = 0, sync_every = 0;  // gk_comm_set_option: the sharded driver's ramp-up and epoch length
    int device = -1;
    bool failed = false;                  // a collective of this communicator returned an error
    std::vector<int> fds;                 // rank 0: fds[r] for r >= 1; others: fds[0] = the link to rank 0
    // RCCL
    Rccl rccl;
    ncclComm_t nc = nullptr;
    hipStream_t stream = nullptr;
    char *dbuf = nullptr;                 // device staging: send block | gathered blocks
    size_t dcap = 0;
    // the shared incumbent words (same host), or null: word (search & 1)
    // serves the current sharded search.  Every rank enters each search of
    // the communicator in the same order, so `search` agrees; a search resets
    // the NEXT search's word at entry, when no rank can be publishing into it
    // (the previous search ended in an all-gather every rank joined, and the
    // next has not begun), so a second glp_intopt on the same communicator
    // never sees the first one's incumbent
    std::atomic<unsigned long long> *inc = nullptr;
    unsigned search = 0;
    ~gk_comm()
    {
        if (inc) (void)munmap((void *)inc, 4096);
        if (nc && rccl.destroy) (void)rccl.destroy(nc);
        if (dbuf) (void)hipFree(dbuf);
        if (stream) (void)hipStreamDestroy(stream);
        for (int fd : fds)
            if (fd >= 0) ::close(fd);
    }
    // the TCP all-gather through rank 0 (also the bootstrap)
    bool tcp_allgather(const void *send, size_t bytes, void *recv)
    {
        char *out = (char *)recv;
        if (rank == 0) {
            std::memcpy(out, send, bytes);
            for (int r = 1; r < size; r++)
                if (!recv_all(fds[r], out + (size_t)r * bytes, bytes)) return false;
            for (int r = 1; r < size; r++)
                if (!send_all(fds[r], out, (size_t)size * bytes)) return false;
            return true;
        }
        return send_all(fds[0], send, bytes) && recv_all(fds[0], out, (size_t)size * bytes);
    }
};

static bool split_addr(const char *addr, std::string &host, int &port)
{
    std::string a = addr ? addr : "";
    const size_t c = a.rfind(':');
    if (c == std::string::npos) return false;
    host = a.substr(0, c);
    if (host.empty()) host = "127.0.0.1";
    port = std::atoi(a.c_str() + c + 1);
    return port > 0 && port < 65536;
}

extern "C" gk_comm *gk_comm_create(gk_ctx *ctx, int rank, int size, const char *addr, int backend)
{
    using gk::set_err;
    if (size < 1 || rank < 0 || rank >= size) { set_err("gk_comm_create: rank %d of %d", rank, size); return nullptr; }
    if (backend != GK_COMM_AUTO && backend != GK_COMM_TCP && backend != GK_COMM_RCCL) {
        set_err("gk_comm_create: backend = %d; invalid", backend);
        return nullptr;
    }
    gk_comm *c = new gk_comm;
    c->rank = rank;
    c->size = size;
    c->device = ctx ? gk_ctx_device(ctx) : -1;
    if (size > 1) {
        std::string host;
        int port = 0;
        if (!split_addr(addr, host, port)) {
            set_err("gk_comm_create: address \"%s\"; expected host:port", addr ? addr : "");
            delete c;
            return nullptr;
        }
        addrinfo hints{}, *ai = nullptr;
        hints.ai_family = AF_INET;
        hints.ai_socktype = SOCK_STREAM;
        if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &ai) != 0 || !ai) {
            set_err("gk_comm_create: cannot resolve %s", host.c_str());
            delete c;
            return nullptr;
        }
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(120);
        bool ok = true;
        if (rank == 0) {
            c->fds.assign(size, -1);
            const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
            int one = 1;
            (void)setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
            timeval tv{120, 0};                   // accept() gives up after 2 minutes
            (void)setsockopt(ls, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
            ok = ls >= 0 && ::bind(ls, ai->ai_addr, ai->ai_addrlen) == 0 && ::listen(ls, size) == 0;
            for (int k = 1; ok && k < size; k++) {
                const int fd = ::accept(ls, nullptr, nullptr);
                int r = -1;
                ok = fd >= 0 && recv_all(fd, &r, sizeof r) && r >= 1 && r < size && c->fds[r] < 0;
                if (ok) {
                    nodelay(fd);
                    c->fds[r] = fd;
                } else if (fd >= 0)
                    ::close(fd);
            }
            if (ls >= 0) ::close(ls);
            if (!ok) set_err("gk_comm_create: rank 0 could not accept the other ranks on %s:%d (%s)", host.c_str(),
                             port, std::strerror(errno));
        } else {
            int fd = -1;
            for (;;) {
                fd = ::socket(AF_INET, SOCK_STREAM, 0);
                if (fd >= 0 && ::connect(fd, ai->ai_addr, ai->ai_addrlen) == 0) break;
                if (fd >= 0) ::close(fd);
                fd = -1;
                if (std::chrono::steady_clock::now() > deadline) break;
                std::this_thread::sleep_for(std::chrono::milliseconds(20));
            }
            ok = fd >= 0 && send_all(fd, &rank, sizeof rank);
            if (ok) {
                nodelay(fd);
                c->fds.assign(1, fd);
            } else {
                if (fd >= 0) ::close(fd);
                set_err("gk_comm_create: rank %d could not reach rank 0 at %s:%d", rank, host.c_str(), port);
            }
        }
        freeaddrinfo(ai);
        if (!ok) {
            delete c;
            return nullptr;
        }
    }
    if (size > 1) {
        // the shared incumbent word, when every rank runs on this host
        char hn[64] = {0};
        (void)gethostname(hn, sizeof hn - 1);
        long long me[2] = {0, (long long)getpid()};
        for (const char *p = hn; *p; ++p) me[0] = me[0] * 131 + *p;
        std::vector<long long> all(2 * size);
        if (!c->tcp_allgather(me, sizeof me, all.data())) {
            set_err("gk_comm_create: bootstrap exchange failed");
            delete c;
            return nullptr;
        }
        bool one_host = true;
        for (int r = 1; r < size; r++) one_host = one_host && all[2 * r] == all[0];
        if (one_host) {
            std::string host;
            int port = 0;
            (void)split_addr(addr, host, port);
            const std::string name = "/gk_inc_" + std::to_string(all[1]) + "_" + std::to_string(port);
            int ok = 1;
            void *p = MAP_FAILED;
            int fd = rank == 0 ? shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600) : -1;
            if (rank == 0) {
                ok = fd >= 0 && ftruncate(fd, 4096) == 0;
                if (ok) p = mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
                ok = ok && p != MAP_FAILED;
                if (ok) {
                    new (p) std::atomic<unsigned long long>(ord_key(DBL_MAX));
                    new ((std::atomic<unsigned long long> *)p + 1) std::atomic<unsigned long long>(ord_key(DBL_MAX));
                }
            }
            std::vector<int> oks(size);
            // rank 0's segment exists (or not) before the others open it
            if (!c->tcp_allgather(&ok, sizeof ok, oks.data())) { delete c; return nullptr; }
            if (rank != 0 && oks[0]) {
                fd = shm_open(name.c_str(), O_RDWR, 0600);
                ok = fd >= 0;
                if (ok) p = mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
                ok = ok && p != MAP_FAILED;
            }
            if (fd >= 0) ::close(fd);
            if (!c->tcp_allgather(&ok, sizeof ok, oks.data())) {
                if (p != MAP_FAILED) (void)munmap(p, 4096);
                if (rank == 0) (void)shm_unlink(name.c_str());
                delete c;
                return nullptr;
            }
            if (rank == 0) (void)shm_unlink(name.c_str());   // every rank has mapped it (or given up)
            const bool every = std::all_of(oks.begin(), oks.end(), [](int v) { return v == 1; });
            if (every) c->inc = (std::atomic<unsigned long long> *)p;
            else if (p != MAP_FAILED) (void)munmap(p, 4096);
        }
    }
    // RCCL when every rank has a device of its own (auto) or when asked; a
    // one-rank communicator takes RCCL only when asked (ncclCommInitRank with
    // nranks = 1 is valid: the transport check of a single process)
    c->backend = GK_COMM_TCP;
    if (size == 1 && backend == GK_COMM_RCCL) {
        ncclUniqueId id;
        if (c->device < 0 || !c->rccl.load() || c->rccl.get_id(&id) != ncclSuccess ||
            hipSetDevice(c->device) != hipSuccess ||
            hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
            c->rccl.init(&c->nc, 1, id, 0) != ncclSuccess) {
            set_err("gk_comm_create: one-rank RCCL communicator could not be created");
            delete c;
            return nullptr;
        }
        c->backend = GK_COMM_RCCL;
    }
    if (size > 1 && backend != GK_COMM_TCP) {
        std::vector<int> devs(size);
        int mine[2] = {c->device, 0};
        // host identity: ranks on different hosts may use the same ordinal
        char hn[64] = {0};
        (void)gethostname(hn, sizeof hn - 1);
        for (const char *p = hn; *p; ++p) mine[1] = mine[1] * 31 + *p;
        std::vector<int> all(2 * size);
        if (!c->tcp_allgather(mine, sizeof mine, all.data())) {
            set_err("gk_comm_create: bootstrap exchange failed");
            delete c;
            return nullptr;
        }
        bool distinct = true;
        for (int r = 0; r < size; r++)
            for (int q = r + 1; q < size; q++)
                if (all[2 * r] < 0 || (all[2 * r] == all[2 * q] && all[2 * r + 1] == all[2 * q + 1])) distinct = false;
        const bool want = backend == GK_COMM_RCCL || distinct;
        if (want && !distinct) {
            set_err("gk_comm_create: RCCL needs one device per rank");
            delete c;
            return nullptr;
        }
        if (want) {
            int have = c->rccl.load() ? 1 : 0;
            std::vector<int> hv(size);
            if (!c->tcp_allgather(&have, sizeof have, hv.data())) { delete c; return nullptr; }
            const bool every = std::all_of(hv.begin(), hv.end(), [](int v) { return v == 1; });
            if (!every && backend == GK_COMM_RCCL) {
                set_err("gk_comm_create: librccl could not be loaded on every rank");
                delete c;
                return nullptr;
            }
            if (every) {
                ncclUniqueId id;
                std::memset(&id, 0, sizeof id);
                if (rank == 0 && c->rccl.get_id(&id) != ncclSuccess) std::memset(&id, 0, sizeof id);
                std::vector<ncclUniqueId> ids(size);
                if (!c->tcp_allgather(&id, sizeof id, ids.data())) { delete c; return nullptr; }
                if (hipSetDevice(c->device) != hipSuccess ||
                    hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
                    c->rccl.init(&c->nc, size, ids[0], rank) != ncclSuccess) {
                    set_err("gk_comm_create: ncclCommInitRank failed on rank %d", rank);
                    delete c;
                    return nullptr;
                }
                c->backend = GK_COMM_RCCL;
            }
        }
    }
    return c;
}

extern "C" void gk_comm_destroy(gk_comm *c) { delete c; }

extern "C" int gk_comm_backend(const gk_comm *c) { return c ? c->backend : -1; }

static int comm_allgather(gk_comm *c, const void *send, size_t bytes, void *recv);

extern "C" int gk_comm_allgather(void *comm, const void *send, size_t bytes, void *recv)
{
    gk_comm *c = (gk_comm *)comm;
    if (!c || (!send && bytes) || (!recv && bytes)) return 1;
    const int r = comm_allgather(c, send, bytes, recv);
    if (r) c->failed = true;
    return r;
}

static int comm_allgather(gk_comm *c, const void *send, size_t bytes, void *recv)
{
    if (c->size == 1 && c->backend != GK_COMM_RCCL) {
        std::memcpy(recv, send, bytes);
        return 0;
    }
    if (c->backend == GK_COMM_TCP) return c->tcp_allgather(send, bytes, recv) ? 0 : 1;
    // RCCL: ncclAllGather on device buffers (xGMI), host blocks in and out
    const size_t need = bytes * (size_t)(c->size + 1);
    if (c->dcap < need) {
        if (c->dbuf) (void)hipFree(c->dbuf);
        c->dbuf = nullptr;
        c->dcap = 0;
        if (hipMalloc((void **)&c->dbuf, need) != hipSuccess) return 1;
        c->dcap = need;
    }
    if (hipSetDevice(c->device) != hipSuccess) return 1;
    char *dsend = c->dbuf, *drecv = c->dbuf + bytes;
    if (hipMemcpyAsync(dsend, send, bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess) return 1;
    if (c->rccl.allgather(dsend, drecv, bytes, ncclChar, c->nc, c->stream) != ncclSuccess) return 1;
    if (hipMemcpyAsync(recv, drecv, bytes * c->size, hipMemcpyDeviceToHost, c->stream) != hipSuccess) return 1;
    return hipStreamSynchronize(c->stream) == hipSuccess ? 0 : 1;
}

extern "C" int gk_comm_rank(const gk_comm *c) { return c ? c->rank : -1; }

namespace gk {
int gk_comm_size_rank(const gk_comm *c, int *rank)
{
    if (rank) *rank = c ? c->rank : 0;
    return c ? c->size : 1;
}

// the column-sharded pricing's exchange (gk_dual.hip lp_shard_trow): RCCL
// on the engine's stream, ordered after the column pass and before the
// pivot's next kernels with no host round trip; TCP (ranks sharing a GPU,
// tests) through the host
int gk_comm_allgather_dev(gk_comm *c, const void *dsend, size_t bytes, void *drecv, hipStream_t s, void *hsend,
                          void *hrecv)
{
    if (!c || c->failed) return 1;
    if (c->backend == GK_COMM_RCCL) {
        if (hipSetDevice(c->device) != hipSuccess) return 1;
        return c->rccl.allgather(dsend, drecv, bytes, ncclChar, c->nc, s) == ncclSuccess ? 0 : 1;
    }
    if (hipMemcpyAsync(hsend, dsend, bytes, hipMemcpyDeviceToHost, s) != hipSuccess) return 1;
    if (hipStreamSynchronize(s) != hipSuccess) return 1;
    if (comm_allgather(c, hsend, bytes, hrecv) != 0) {
        c->failed = true;
        return 1;
    }
    return hipMemcpyAsync(drecv, hrecv, bytes * (size_t)c->size, hipMemcpyHostToDevice, s) == hipSuccess ? 0 : 1;
}

// a rank-local failure inside a collective sequence (the sharded LP): the
// communicator is marked failed and its links are shut down, so that every
// peer's next exchange returns an error instead of waiting for this rank
// (their failure then shuts their own links: the abort reaches every rank)
void gk_comm_abort(gk_comm *c)
{
    if (!c) return;
    c->failed = true;
    for (int fd : c->fds)
        if (fd >= 0) (void)::shutdown(fd, SHUT_RDWR);
    if (c->nc && c->rccl.abort) {
        (void)c->rccl.abort(c->nc);
        c->nc = nullptr;
    }
}
bool shard_any(LpShard &sh, bool flag)
{
    const char mine = flag ? 1 : 0;
    std::vector<char> all((size_t)sh.size, 0);
    if (sh.failed || gk_comm_allgather(sh.comm, &mine, 1, all.data()) != 0) {
        sh.failed = true;
        throw std::runtime_error("column-sharded pricing: the stop decision's exchange failed");
    }
    for (char c : all)
        if (c) return true;
    return false;
}

void shard_abort(LpShard &sh)
{
    sh.failed = true;
    gk_comm_abort(sh.comm);
}
}  // namespace gk

extern "C" double gk_comm_incumbent(gk_comm *c, double mine)
{
    if (!c || !c->inc) return mine;
    std::atomic<unsigned long long> *w = c->inc + (c->search & 1);
    const unsigned long long k = ord_key(mine);
    unsigned long long cur = w->load(std::memory_order_relaxed);
    while (k < cur && !w->compare_exchange_weak(cur, k, std::memory_order_acq_rel)) {}
    return ord_val(std::min(k, w->load(std::memory_order_acquire)));
}

extern "C" int gk_comm_shared_incumbent(const gk_comm *c) { return c && c->inc ? 1 : 0; }

extern "C" int gk_comm_set_option(gk_comm *c, int opt, int value)
{
    if (!c) return GK_EABI;
    if (opt == GK_COMM_OPT_RAMP) c->ramp_nodes = value;
    else if (opt == GK_COMM_OPT_SYNC) c->sync_every = value;
    else { gk::set_err("gk_comm_set_option: opt = %d; invalid", opt); return GK_EABI; }
    return 0;
}
extern "C" int gk_comm_size(const gk_comm *c) { return c ? c->size : -1; }

// glp_intopt over every rank of comm: the sharded search
// (gk_ios_driver_sharded with this library's all-gather), then one more
// all-gather that agrees on the winning incumbent — the best objective,
// the lowest rank on ties — so every rank returns the same solution
extern "C" int gk_ios_driver_comm(gk_ctx *ctx, gk_mip *mip, const gk_iocp *parm, gk_comm *comm)
{
    using gk::set_err;
    if (!comm) { set_err("gk_ios_driver_comm: null communicator"); return GK_EABI; }
    if (comm->size == 1 && comm->backend != GK_COMM_RCCL) return gk_ios_driver(ctx, mip, parm);
    // this search's incumbent word (gk_comm::inc); the next one's is cleared
    struct SearchScope {
        gk_comm *c;
        explicit SearchScope(gk_comm *cc) : c(cc)
        {
            if (c->inc) c->inc[(c->search + 1) & 1].store(ord_key(DBL_MAX), std::memory_order_relaxed);
        }
        ~SearchScope() { c->search++; }
    } scope(comm);
    gk_ios_shard sh{};
    sh.rank = comm->rank;
    sh.size = comm->size;
    sh.ramp_nodes = comm->ramp_nodes;
    sh.sync_every = comm->sync_every;
    sh.exchange = nullptr;
    sh.info = comm;
    sh.allgather = gk_comm_allgather;
    // the shared incumbent word between the epochs (ranks on one host)
    auto inc = [](void *info, double mine) { return gk_comm_incumbent((gk_comm *)info, mine); };
    const int ret = gk_ios_driver_sharded_inc(ctx, mip, parm, &sh, comm->inc ? +inc : nullptr, comm);
    // a local failure inside the search reaches the other ranks through the
    // sync epoch (every rank leaves the search together); this rank still
    // joins the final all-gather, with its error in h[2], so that no peer
    // waits for it.  After a failed collective the sequence is lost: return.
    if (ret == GK_EABI && comm->failed) return ret;
    std::string my_err;
    if (ret == GK_EABI) my_err = gk_last_error();
    const int m = mip->lp.m, n = mip->lp.n;
    const size_t blk = 4 * sizeof(double) + ((size_t)m + n) * sizeof(double);
    std::vector<char> me(blk, 0), all(blk * comm->size);
    double *h = (double *)me.data();
    const bool have = mip->mip_stat == 5 || mip->mip_stat == 2;      // GLP_OPT / GLP_FEAS
    h[0] = have ? 1.0 : 0.0;
    h[1] = have ? mip->mip_obj : 0.0;
    h[2] = (double)ret;
    h[3] = (double)mip->mip_stat;
    for (int i = 0; i < m; i++) h[4 + i] = mip->row_mipx[i + 1];
    for (int j = 0; j < n; j++) h[4 + m + j] = mip->col_mipx[j + 1];
    if (gk_comm_allgather(comm, me.data(), blk, all.data()) != 0) {
        set_err("gk_ios_driver_comm: final all-gather failed");
        return GK_EABI;
    }
    if (ret == GK_EABI) {
        set_err("%s", my_err.c_str());
        return ret;
    }
    for (int r = 0; r < comm->size; r++)
        if ((int)((const double *)(all.data() + (size_t)r * blk))[2] == GK_EABI) {
            set_err("gk_ios_driver_comm: rank %d failed", r);
            return GK_EABI;
        }
    const double sign = (mip->lp.dir == 1) ? 1.0 : -1.0;               // GLP_MIN
    int win = -1, worst_ret = 0;
    bool any_partial = false;
    for (int r = 0; r < comm->size; r++) {
        const double *g = (const double *)(all.data() + (size_t)r * blk);
        if ((int)g[2] != 0) worst_ret = (int)g[2];
        if ((int)g[3] == 2 || (int)g[3] == 1) any_partial = true;   // stopped before proving optimality
        if (g[0] != 1.0) continue;
        if (win < 0 || sign * g[1] < sign * ((const double *)(all.data() + (size_t)win * blk))[1]) win = r;
    }
    if (win >= 0) {
        const double *g = (const double *)(all.data() + (size_t)win * blk);
        mip->mip_obj = g[1];
        for (int i = 0; i < m; i++) mip->row_mipx[i + 1] = g[4 + i];
        for (int j = 0; j < n; j++) mip->col_mipx[j + 1] = g[4 + m + j];
        mip->mip_stat = (worst_ret == 0 && !any_partial) ? 5 : 2;
    } else {
        mip->mip_obj = 0.0;
        mip->mip_stat = (worst_ret == 0 && !any_partial) ? 4 : 1;
    }
    return worst_ret;
}
