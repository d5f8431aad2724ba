// engine.cpp -- host runtime of the hdpm MI355X engine and its C ABI (include/hdpm.h).
//
// Owns the device-resident chain state and drives the gfx950 kernels in kernels.hip.
// The host keeps the single R-compatible random stream and performs the draws that
// consume a data-dependent number of uniforms (update_phi's center/sigma draws, pool
// generation); the device consumes contiguous (m+1)-per-point slices for the sweep.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cctype>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <pthread.h>
#include <sched.h>
#include <dirent.h>
#include <dlfcn.h>
#include <execinfo.h>
#include <csignal>
#include <unistd.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/hdpm.h"
#include "host_topology.hpp"
#include "kernels.hpp"
#include "mtjump.hpp"
#include "pool_host.hpp"
#include "rmath.hpp"

namespace hdpm {

hipError_t launch_prepass(const PrepassArgs& a, int nblocks, hipStream_t s);
hipError_t launch_cluster_summary(const PrepassArgs& a, hipStream_t s);
hipError_t launch_dense_list(const PrepassArgs& a, hipStream_t s);
hipError_t launch_resolve(const ResolveArgs& a, hipStream_t s);
hipError_t launch_exact_rows(const PrepassArgs& a, int nblocks, hipStream_t s, int* path = nullptr);
size_t resolve_smem_bytes(int scap, int m, int blocks);
size_t resolve_fpg_smem_bytes(int lcap, int m);
int resolve_fpg_max_grid(int lcap, int m);
int warm_sweep_kernels(int lcap, int m);
hipError_t warm_launch_kernels(const PrepassArgs& pa, const ResolveArgs& ra, const int* zero, int* scratch,
                               hipStream_t s);
int device_cus();
hipError_t launch_relabel(int* c, const int* los, int n, const ResolveCtl* ctl, hipStream_t s);
hipError_t launch_finish_sweep(int* counts, int* sol, int* los, int* src, int cap, const ResolveCtl* ctl, int n,
                               hipStream_t s);
hipError_t launch_apply_moves(const int* mlog, const int* mcount, int grid, const uint8_t* codes_t, int d, int nq,
                              int mmax, unsigned int* freq, const ResolveCtl* ctl, int n, int nslots, hipStream_t s);
hipError_t launch_freq_gather(const unsigned int* freq, const int* sol, int Kmax, int fs, unsigned int* out,
                              const ResolveCtl* ctl, int n, hipStream_t s);
hipError_t launch_scatter_clusters(const uint8_t* stage, int nent, int dp, int d, int bw, int full, uint8_t* codes,
                                   double* tab, uint64_t* bnd, int* counts, int* sol, int* los, int* src,
                                   hipStream_t s, const int* gate = nullptr, uint64_t* csum = nullptr,
                                   const double* logn = nullptr, int* zero = nullptr, int* wide_ctr = nullptr);
hipError_t launch_phi_locate(const PipeArgs& a, hipStream_t s);
hipError_t launch_pipe_wait(PipeSlot* slot, const ResolveCtl* prev, ResolveCtl* own, int n, PipeGate* g,
                            long long limit, hipStream_t s, const PipeAuto& au);
hipError_t launch_pipe_check(const PipeArgs& a, hipStream_t s);
hipError_t launch_pool_heads(const double* tab, const uint64_t* bnd, int64_t P, int d, int wb, int Ws, int bw, int ha,
                             int hb, uint64_t* head, hipStream_t s);
hipError_t launch_hist(const HistArgs& a, hipStream_t s);
size_t hist_partial_words(const HistArgs& a, int* nbx, int* kc, int* tpb);
hipError_t launch_loglik(const LoglikArgs& a, hipStream_t s);
hipError_t launch_mt_gen(const MtGenArgs& a, hipStream_t s);
hipError_t launch_psm(const int32_t* trace, int M, int N, uint8_t* lab, uint32_t* cnt, hipStream_t s);
hipError_t launch_vi_terms(const uint32_t* cnt, int N, int M, const int32_t* cls, int ncand, double* all, double* same,
                           hipStream_t s);
hipError_t launch_debug_draw(const double* logw, int E, double rU, int two_way, int ocml, int* out, hipStream_t s);
hipError_t launch_debug_math(const double* x, int64_t n, int fn, int ocml, double* out, hipStream_t s);
hipError_t launch_lmatrix(const uint8_t* codes_t, int n, int d, int nq, ParamTables cl, int K, double* L,
                          int* H, int64_t ldL, hipStream_t s);
hipError_t launch_phi(const PhiArgs& a, hipStream_t s);
hipError_t launch_phi2(const PhiArgs& a, hipStream_t s, hipEvent_t before_values = nullptr);
size_t phi2_group_lds_bytes(int gs, int nw, double rate);
size_t phi2_tree_lds_bytes(int T, int G, int tW);
size_t phi2_values_lds_bytes(int d, int G, int tW, int T);
size_t phi_cwalk_lds(int d, int nw, int wpb);
size_t phi_values_lds(int d, int nw);
size_t phi_tree_lds_bytes(int SB, int nw, int W);
size_t phi_values2_lds_bytes(int d, int nb, int T, int W, int nw);
int phi_ilp();
int sm_restricted_gibbs_device(struct Ctx* c, const int32_t* S, int32_t nS, int32_t i1, int32_t i2,
                               int32_t t);

struct HipError {
  hipError_t e;
  const char* what;
};
#define HIPCHK(x)                                      \
  do {                                                 \
    hipError_t _e = (x);                               \
    if (_e != hipSuccess) throw HipError{_e, #x};     \
  } while (0)

#ifndef HDPM_PHI_SPEC
#define HDPM_PHI_SPEC 4   // update_phi phase B: first rbeta attempts speculated per batch
#endif
static std::atomic<int64_t> g_dev_allocs{0};   // device allocations made (diagnostics)

// HDPM_SEGV_TRACE=1: a host fault prints the raw return addresses of the faulting stack and
// the library's load address (for addr2line), then hands the signal to the handler that was
// installed before (Python's faulthandler, a runtime's), or to the default action.  Only
// async-signal-safe calls in the handler: the frames are walked by backtrace() and written
// by backtrace_symbols_fd() (both preloaded at install time, so no allocation or dynamic
// loading happens in the handler), the text by write().
static struct sigaction g_segv_prev;
static uintptr_t g_lib_base = 0;
static void segv_put_hex(uintptr_t x) {
  char buf[32];
  int k = 0;
  buf[k++] = '0';
  buf[k++] = 'x';
  char tmp[16];
  int t = 0;
  do { tmp[t++] = "0123456789abcdef"[x & 15]; x >>= 4; } while (x && t < 16);
  while (t) buf[k++] = tmp[--t];
  buf[k++] = '\n';
  (void)!write(2, buf, (size_t)k);
}
static void segv_trace(int sig, siginfo_t* info, void* uctx) {
  static const char hdr[] = "libhdpm: fault; library base ";
  (void)!write(2, hdr, sizeof(hdr) - 1);
  segv_put_hex(g_lib_base);
  void* fr[64];
  const int nf = backtrace(fr, 64);
  backtrace_symbols_fd(fr, nf, 2);
  if (g_segv_prev.sa_flags & SA_SIGINFO) {
    if (g_segv_prev.sa_sigaction) { g_segv_prev.sa_sigaction(sig, info, uctx); return; }
  } else if (g_segv_prev.sa_handler != SIG_DFL && g_segv_prev.sa_handler != SIG_IGN && g_segv_prev.sa_handler) {
    g_segv_prev.sa_handler(sig);
    return;
  }
  // default action: re-raised with the default disposition on return from the handler
  struct sigaction dfl;
  std::memset(&dfl, 0, sizeof(dfl));
  dfl.sa_handler = SIG_DFL;
  sigemptyset(&dfl.sa_mask);
  sigaction(sig, &dfl, nullptr);
  raise(sig);
}
static const bool g_segv_trace = [] {
  if (!std::getenv("HDPM_SEGV_TRACE")) return false;
  Dl_info di;
  if (dladdr((void*)&segv_put_hex, &di)) g_lib_base = (uintptr_t)di.dli_fbase;
  void* warm[2];
  (void)backtrace(warm, 2);          // loads libgcc's unwinder now, not inside the handler
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = segv_trace;
  sa.sa_flags = SA_SIGINFO;
  sigemptyset(&sa.sa_mask);
  return sigaction(SIGSEGV, &sa, &g_segv_prev) == 0;
}();

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  // Grow to at least `count` elements; keep_old copies the previous contents.
  void ensure(size_t count, bool keep_old = false, hipStream_t s = nullptr) {
    if (count <= n && p) return;
    T* np = nullptr;
    g_dev_allocs.fetch_add(1, std::memory_order_relaxed);
    HIPCHK(hipMalloc(&np, std::max<size_t>(count, 1) * sizeof(T)));
    if (keep_old && p && n) {
      HIPCHK(hipMemcpyAsync(np, p, n * sizeof(T), hipMemcpyDeviceToDevice, s));
      HIPCHK(hipStreamSynchronize(s));
    }
    release();
    p = np;
    n = count;
  }
};

template <class T>
struct PinBuf {
  T* p = nullptr;
  size_t n = 0;
  ~PinBuf() {
    if (p) (void)hipHostFree(p);
  }
  // non-coherent (coarse-grained) by default: CPU-cached, so the host reads these buffers
  // at cache speed; every device write to them is followed by a stream or event wait
  // before use.  Buffers kernels read or write in place (no copy) are coherent.
  void ensure(size_t count, unsigned flags = hipHostMallocNonCoherent) {
    if (count <= n && p) return;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    HIPCHK(hipHostMalloc(&p, std::max<size_t>(count, 1) * sizeof(T), flags));
    n = count;
  }
};

static int host_threads() {
  unsigned h = std::thread::hardware_concurrency();
  if (h == 0) h = 4;
  return (int)std::min<unsigned>(h, 16);
}

template <class F>
static void parallel_for(int64_t n, F f) {
  const int T = host_threads();
  if (n < 4096 || T <= 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> th;
  const int64_t chunk = (n + T - 1) / T;
  for (int t = 0; t < T; ++t) {
    int64_t a = t * chunk, b = std::min(n, a + chunk);
    if (a >= b) break;
    th.emplace_back([=] { f(a, b); });
  }
  for (auto& x : th) x.join();
}

// CPU list files of sysfs ("0-7,16-23").
static std::vector<int> read_cpu_list(const std::string& path) {
  std::vector<int> out;
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) return out;
  char buf[4096];
  if (!std::fgets(buf, sizeof(buf), f)) buf[0] = 0;
  std::fclose(f);
  for (char* p = buf; *p;) {
    char* end;
    long a = std::strtol(p, &end, 10);
    if (end == p) { ++p; continue; }
    long b = a;
    if (*end == '-') b = std::strtol(end + 1, &end, 10);
    for (long c = a; c <= b; ++c) out.push_back((int)c);
    p = end;
  }
  return out;
}

// Persistent host worker pool for the per-iteration host phases (the deterministic parts
// of the parameter draws, table builds).  Workers spin for a short while after a job and
// then sleep; prewake() gets sleeping workers spinning ahead of a job (e.g. while the
// host waits for the device), so dispatch costs about a microsecond.
// HDPM_HOST_THREADS sets the number of threads (default min(8, hardware threads)),
// HDPM_SPIN_US the spin window.
class HostPool {
 public:
  // The pool of the calling engine call's context (PoolScope), else, on a pool worker, its
  // own pool, else the process's default pool (the creating thread's L3 domain).
  static HostPool& get() {
    if (HostPool* p = current()) return *p;
    return for_home(std::vector<int>{});
  }
  // One pool per home L3 domain (created on first use, alive for the process): contexts
  // whose GPUs have different homes get different pools (gpu_home_domain).
  static HostPool& for_home(const std::vector<int>& dom) {
    static std::mutex mu;
    static std::vector<std::pair<std::vector<int>, std::unique_ptr<HostPool>>> pools;
    std::lock_guard<std::mutex> lk(mu);
    for (auto& e : pools)
      if (e.first == dom) return *e.second;
    pools.emplace_back(dom, std::unique_ptr<HostPool>(new HostPool(dom)));
    return *pools.back().second;
  }
  static HostPool*& current() {
    static thread_local HostPool* p = nullptr;
    return p;
  }
  int threads() const { return (int)th_.size() + 1; }
  int workers() const { return (int)th_.size(); }

  // f(lo, hi) over [0, n) in chunks of `grain` on all threads; returns when done.
  template <class F>
  void run(int64_t n, int64_t grain, F&& f) {
    if (n <= 0) return;
    if (th_.empty() || n <= grain) {
      f((int64_t)0, n);
      return;
    }
    // another context's job still open on the pool (its try_launch() holds the pool across
    // API calls, possibly on this same thread): run on the calling thread instead of waiting
    if (!acquire()) {
      f((int64_t)0, n);
      return;
    }
    struct Release {
      HostPool* p;
      ~Release() { p->busy_.store(false, std::memory_order_release); }
    } rel{this};
    quiesce();
    // a worker that saw the last generation but registers only now finds nothing to take
    // while the job's fields are rewritten (next_ past any total, launches closed)
    next_.store(INT64_MAX / 2, std::memory_order_release);
    bclaim_.store(kClosed, std::memory_order_release);
    range_ = [&f](int64_t a, int64_t b) { f(a, b); };
    bcast_ = nullptr;
    total_ = n;
    grain_ = grain;
    done_.store(0, std::memory_order_relaxed);
    next_.store(0, std::memory_order_release);
    publish();
    work();
    while (done_.load(std::memory_order_acquire) < total_) spin_pause();
  }

  // Workers that wake up while the job is open call f(worker_index) once; the caller
  // continues.  join() closes the job and waits only for the workers that joined it, so a
  // worker the OS has not run yet (a busy core) holds nobody up: f must hand out its work
  // through shared counters that the caller drains too.
  // false (nothing launched) while another context's job holds the pool: the caller then
  // drains its job alone, which every launched job supports
  template <class F>
  bool try_launch(F&& f) {
    if (!acquire()) return false;
    quiesce();
    bclaim_.store(kClosed, std::memory_order_release);     // (see run)
    next_.store(INT64_MAX / 2, std::memory_order_release);
    bjob_ = std::forward<F>(f);
    bcast_ = &bjob_;
    range_ = nullptr;
    bdone_.store(0, std::memory_order_relaxed);
    bclaim_.store(0, std::memory_order_release);
    publish();
    return true;
  }
  void join() {
    const int joined = bclaim_.fetch_or(kClosed, std::memory_order_acq_rel) & ~kClosed;
    while (bdone_.load(std::memory_order_acquire) < joined) spin_pause();
    busy_.store(false, std::memory_order_release);
  }

  void prewake() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      wake_seq_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
  }

  static void spin_pause() { __builtin_ia32_pause(); }

  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }

 private:
  explicit HostPool(const std::vector<int>& home) : home_(home) {
    if (const char* e = std::getenv("HDPM_SPIN_US")) spin_us_ = std::max(0, std::atoi(e));
    int T = 0;
    if (const char* e = std::getenv("HDPM_HOST_THREADS")) T = std::atoi(e);
    if (T <= 0) {
      unsigned h = std::thread::hardware_concurrency();
      T = (int)std::min<unsigned>(h ? h : 4, 8);
    }
    for (int t = 1; t < T; ++t)
      th_.emplace_back([this] {
        current() = this;        // jobs running on a worker see their own pool
        loop();
      });
    pin_workers();
  }
  // Workers on distinct physical cores of one L3 domain (the host phases hand data between
  // cores every iteration): the pool's home domain (the GPU's, hdpm_ctx_create), else the
  // creating thread's; HDPM_PIN_THREADS=0 leaves placement to the OS.
  void pin_workers() {
    if (const char* e = std::getenv("HDPM_PIN_THREADS"))
      if (std::atoi(e) == 0) return;
    cpu_set_t allowed;
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return;
    const std::string base = "/sys/devices/system/cpu/cpu";
    std::vector<int> dom = home_;
    int me = dom.empty() ? sched_getcpu() : dom.front();
    if (me < 0) return;
    main_cpu_ = me;
    if (dom.empty()) dom = read_cpu_list(base + std::to_string(me) + "/cache/index3/shared_cpu_list");
    if (dom.empty()) return;
    auto read_list = [](const std::string& path) { return read_cpu_list(path); };
    std::vector<char> used_core(4096, 0);
    auto core_of = [&](int c) {
      const std::vector<int> sib = read_list(base + std::to_string(c) + "/topology/thread_siblings_list");
      return sib.empty() ? c : sib.front();
    };
    used_core[core_of(me) & 4095] = 1;
    std::vector<int> pick;
    for (int c : dom) {
      if (!CPU_ISSET(c, &allowed)) continue;
      const int core = core_of(c) & 4095;
      if (used_core[core]) continue;
      used_core[core] = 1;
      pick.push_back(c);
    }
    for (size_t t = 0; t < th_.size() && t < pick.size(); ++t) {
      cpu_set_t cs;
      CPU_ZERO(&cs);
      CPU_SET(pick[t], &cs);
      (void)pthread_setaffinity_np(th_[t].native_handle(), sizeof(cs), &cs);
    }
  }
  void quiesce() {
    while (active_.load(std::memory_order_acquire) != 0) spin_pause();
  }
  // The pool is owned by one job at a time: a flag taken by compare-and-swap (not a mutex --
  // a launched job holds it across API calls and may be joined from another thread).
  bool acquire() {
    bool expect = false;
    return busy_.compare_exchange_strong(expect, true, std::memory_order_acq_rel);
  }
  void publish() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
  }
  void work() {
    for (;;) {
      const int64_t a = next_.fetch_add(grain_, std::memory_order_acquire);
      if (a >= total_) break;
      const int64_t b = std::min(total_, a + grain_);
      range_(a, b);
      done_.fetch_add(b - a, std::memory_order_release);
    }
  }
  void loop() {
    uint64_t seen = 0, woke = 0;
    for (;;) {
      auto t0 = std::chrono::steady_clock::now();
      int polls = 0;
      for (;;) {
        // spin on the generation with plain loads (registering in active_ on every poll kept
        // its cache line bouncing between the cores and stalled quiesce()); register, then
        // look again, only when it changed
        if (gen_.load(std::memory_order_acquire) == seen) {
          if (stop_) return;
          spin_pause();
          if (++polls % 256 == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_)) {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] {
              return stop_ || gen_.load(std::memory_order_acquire) != seen ||
                     wake_seq_.load(std::memory_order_acquire) != woke;
            });
            woke = wake_seq_.load(std::memory_order_acquire);
            if (stop_) return;
            t0 = std::chrono::steady_clock::now();
          }
          continue;
        }
        active_.fetch_add(1, std::memory_order_acq_rel);
        const uint64_t g = gen_.load(std::memory_order_acquire);
        if (g != seen) {
          seen = g;
          if (bcast_) {
            const int id = bclaim_.fetch_add(1, std::memory_order_acq_rel);
            if (!(id & kClosed)) {
              (*bcast_)(id);
              bdone_.fetch_add(1, std::memory_order_acq_rel);
            }
          } else {
            work();
          }
          active_.fetch_sub(1, std::memory_order_acq_rel);
          break;
        }
        active_.fetch_sub(1, std::memory_order_acq_rel);
        if (stop_) return;
        spin_pause();
        if (++polls % 256 == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_)) {
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [&] {
            return stop_ || gen_.load(std::memory_order_acquire) != seen ||
                   wake_seq_.load(std::memory_order_acquire) != woke;
          });
          woke = wake_seq_.load(std::memory_order_acquire);
          if (stop_) return;
          t0 = std::chrono::steady_clock::now();
        }
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::atomic<bool> busy_{false};
  std::condition_variable cv_;
  std::atomic<uint64_t> gen_{0}, wake_seq_{0};
  static constexpr int kClosed = 1 << 30;
  std::atomic<int> active_{0}, bdone_{0}, bclaim_{0};
  std::atomic<int64_t> next_{0}, done_{0};
  int64_t total_ = 0, grain_ = 1;
  std::function<void(int64_t, int64_t)> range_;
  std::function<void(int)> bjob_;
  std::function<void(int)>* bcast_ = nullptr;
  std::atomic<bool> stop_{false};
  int spin_us_ = 2000;   // an iteration's host phases are ~1 ms apart: stay awake between them
  int main_cpu_ = -1;    // the calling thread's core (kept free of workers)
  std::vector<int> home_;   // CPUs of the L3 domain the pool lives on (empty: the creator's)

 public:
  int main_cpu() const { return main_cpu_; }
  const std::vector<int>& home() const { return home_; }
};

// The context's pool for the duration of an engine call (C ABI entry points).
struct PoolScope {
  HostPool* prev;
  explicit PoolScope(HostPool* p) : prev(HostPool::current()) {
    if (p) HostPool::current() = p;
  }
  ~PoolScope() { HostPool::current() = prev; }
};

// The host pool's home for a process driving `device`: an L3 domain among the CPUs local to
// the GPU (its PCI device's local_cpulist, within this process's affinity), a different
// one for each GPU that shares those CPUs, so one process per GPU (bench.py --gpus N)
// spreads its pinned workers instead of stacking them on whichever domain each process
// started on.  Empty (creating thread's domain) when the topology is not readable.
static std::vector<int> gpu_home_domain(int device) {
  std::vector<int> none;
  if (const char* e = std::getenv("HDPM_PIN_THREADS"))
    if (std::atoi(e) == 0) return none;
  int cnt = 0;
  if (hipGetDeviceCount(&cnt) != hipSuccess || device < 0 || device >= cnt) return none;
  auto local_list = [](int dev) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) != hipSuccess) return std::vector<int>{};
    for (char* p = bus; *p; ++p) *p = (char)std::tolower((unsigned char)*p);
    return read_cpu_list(std::string("/sys/bus/pci/devices/") + bus + "/local_cpulist");
  };
  const std::vector<int> mine = local_list(device);
  if (mine.empty()) return none;
  int slot = 0, share = 0;
  // this GPU's rank among all the node's AMD accelerators with the same local CPUs (sysfs:
  // also the ones this process cannot see, so processes on different GPUs of a node pick
  // different domains even when each sees only its own), else among the visible ones
  {
    char bus[64] = {0};
    std::vector<std::string> peers;
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) == hipSuccess) {
      for (char* p = bus; *p; ++p) *p = (char)std::tolower((unsigned char)*p);
      if (DIR* dir = opendir("/sys/bus/pci/devices")) {
        while (dirent* e = readdir(dir)) {
          if (e->d_name[0] == '.') continue;
          const std::string dev = std::string("/sys/bus/pci/devices/") + e->d_name;
          char vendor[16] = {0}, cls[16] = {0};
          FILE* f = std::fopen((dev + "/vendor").c_str(), "r");
          if (!f) continue;
          const bool okv = std::fgets(vendor, sizeof(vendor), f) != nullptr;
          std::fclose(f);
          f = std::fopen((dev + "/class").c_str(), "r");
          if (!f) continue;
          const bool okc = std::fgets(cls, sizeof(cls), f) != nullptr;
          std::fclose(f);
          if (!okv || !okc || std::strncmp(vendor, "0x1002", 6) != 0) continue;
          if (std::strncmp(cls, "0x1200", 6) != 0 && std::strncmp(cls, "0x0380", 6) != 0) continue;
          if (read_cpu_list(dev + "/local_cpulist") == mine) peers.push_back(e->d_name);
        }
        closedir(dir);
      }
    }
    std::sort(peers.begin(), peers.end());
    for (size_t q = 0; q < peers.size(); ++q)
      if (peers[q] == bus) {
        slot = (int)q;
        share = (int)peers.size();
      }
  }
  if (share == 0)
    for (int d2 = 0; d2 < cnt; ++d2)
      if (local_list(d2) == mine) {
        if (d2 < device) ++slot;
        ++share;
      }
  cpu_set_t allowed;
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return none;
  return choose_home_domain(
      mine, slot, share,
      [](int c) {
        const std::vector<int> l3 =
            read_cpu_list("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/cache/index3/shared_cpu_list");
        return l3.empty() ? c : l3.front();
      },
      [&](int c) { return c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &allowed); });
}

// The calling thread on the core kept free of pool workers for the duration of an engine
// call (the serial draws share data with the workers through the L3); the caller's
// affinity is restored on exit.  HDPM_PIN_THREADS=0 disables it.
struct ScopedPin {
  cpu_set_t old;
  bool active = false;
  ScopedPin() {
    const int c = HostPool::get().main_cpu();
    if (c < 0 || sched_getaffinity(0, sizeof(old), &old) != 0 || !CPU_ISSET(c, &old)) return;
    cpu_set_t cs;
    CPU_ZERO(&cs);
    CPU_SET(c, &cs);
    active = sched_setaffinity(0, sizeof(cs), &cs) == 0;
  }
  ~ScopedPin() {
    if (active) (void)sched_setaffinity(0, sizeof(old), &old);
  }
};

template <class F>
static void pool_for(int64_t n, F f, int64_t grain = 0) {
  HostPool& P = HostPool::get();
  if (grain <= 0) grain = std::max<int64_t>(1, n / (4 * P.threads()));
  P.run(n, grain, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) f((int)i);
  });
}

// Device scratch of the split-merge move (split_merge.inl).
struct SmWork {
  DevBuf<int> d_S, d_side, d_side_ref, d_counts2, d_cert, d_side_prev;
  DevBuf<double> d_ll, d_out;
  DevBuf<uint8_t> d_two_codes;
  DevBuf<double> d_two_tab;
  DevBuf<uint32_t> d_raw;
  std::vector<double> h_out;
  // pinned staging of the restricted scans' per-iteration transfers (sides, draws, tables)
  PinBuf<int> h_side;
  PinBuf<uint32_t> h_raw;
  PinBuf<uint8_t> h_two_codes;
  PinBuf<double> h_two_tab;
  DevBuf<int> d_wide;         // k_sm_scan_wide's barrier, flags and chunk deltas
  PinBuf<int> h_wide;
  DevBuf<uint32_t> d_freq;    // k_sm_freq's table
  PinBuf<uint32_t> h_freq;
  // norm_const2(w_j, v_j, m_j) of the prior density (sm:419-436 priors): a function of the
  // hyperparameters alone, computed once per (v, w, log-space mode)
  std::vector<double> prior_nc, prior_v, prior_w;
  std::vector<int32_t> prior_att;
  std::vector<int> prior_err;
  int prior_log = -1;
  int64_t phi_prefetch = 0;   // stream slice generated ahead for the move's update_phi jobs
  // the restricted Gibbs sampler's device chain (split_merge.inl sm_chain), by scan k
  DevBuf<SmLink> d_links;
  DevBuf<PhiChain> d_chain;   // [0] the seed (the chain's first position), then per scan the link's (1 + 2k) and the update's (2 + 2k)
  DevBuf<uint32_t> d_F, d_FM; // both tables (ascending label order); the table of S + {i1, i2}
  DevBuf<int> d_labcnt, d_labdev;   // [k][4] each update's labels and sizes (k_sm_tabs), their copy (k_phi2_group)
  DevBuf<uint8_t> d_stage;    // [k] each update's staged tables
  DevBuf<double> d_sig;       // [k + 1][2 d] sigmas: the chain's first, then each update's
  PinBuf<uint8_t> h_cout;     // [k] each update's outputs, status and stream state (coherent)
  PinBuf<uint8_t> h_cin, h_cback;   // the chain's inputs; its results (tables, chain words, scan flags)
  hipEvent_t ev_chain = nullptr;
};

// A window of the R random stream generated on the device (k_mt_gen), starting at the
// host stream position start_pos.  Two windows alternate: while a sweep consumes one, the
// next window is generated from the state where that sweep's draws end, so the device
// generator runs concurrently with the sweep and the host-side update_phi draws.
struct RngWindow {
  DevBuf<uint32_t> raw, arrays, init;
  const uint32_t* init_src = nullptr;   // initial array on the device (init.p or a block of another window)
  PinBuf<uint32_t> h_init;
  uint64_t start_pos = 0, epoch = ~0ull;
  int64_t count = 0;
  int mti0 = 624, nblocks = 0, export_from = 1;
  int64_t export_after = 0;
  hipEvent_t done = nullptr;
  bool valid = false;
  uint64_t gen = 0;                     // launches of this window (a pipelined sweep waited on one)
};

struct Ctx {
  int device = 0;
  HostPool* hpool = nullptr;       // the host worker pool homed next to this GPU (HostPool::for_home)
  hipStream_t stream = nullptr;
  hipStream_t gstream = nullptr;   // random-stream generator
  hipStream_t cstream = nullptr;   // copies of stream states to the host (never queued behind a generator launch)
  hipStream_t pstream = nullptr;   // update_phi speculated on the device beside the sweep (dspec)
  // update_phi's slice of the stream copied from the window that holds it (StreamAhead::fill_raw)
  struct PhiDev {
    bool valid = false;
    uint64_t pos = 0, epoch = 0;
    int mti = 0;
    int64_t N = 0;
    hipEvent_t ev = nullptr;           // the copy of the slice holding it
    const uint32_t* blk = nullptr;     // tempered words from the start of the state's block
  } phidev;
  // Host copies of stretches of the device windows (a ring): the slice of the next update,
  // or one fetched an iteration ahead (phi_lookahead) so that the next one needs no copy.
  struct PhiSlice {
    PinBuf<uint32_t> buf;
    hipEvent_t ev = nullptr;
    uint64_t s0 = 0, epoch = ~0ull, stamp = 0;
    int64_t words = 0;
    bool valid = false;
  } phis[3];
  uint64_t phis_clock = 0;
  uint64_t look_from = 0;              // the stretch the next lookahead copies (0: none)
  int64_t look_words = 0;
  RngWindow win[2];
  // MT jump-ahead for multi-workgroup windows (mtjump.hpp)
  int mt_G = 0, mt_bpg = 0;
  DevBuf<uint64_t> d_jpoly;
  DevBuf<uint32_t> d_jidx;
  DevBuf<int> d_joff;
  int64_t cmax = 1 << 16;          // draws expected between two sweeps (update_phi etc.)
  // Host-state adoption in flight: rng.pos is current, rng.mt / rng.mti arrive with `ev`
  // (rng_sync() before any host use of the stream).
  struct PendingAdopt {
    bool active = false;
    hipEvent_t ev = nullptr;
    PinBuf<uint32_t> arr;
    const uint32_t* host_src = nullptr;
    const uint32_t* from_raw = nullptr;   // tempered words of the state's block (phi_device_prefetch)
    int mti = 0;
  } pend;
  std::string err;
  hipEvent_t ev[8];

  // aux_data
  int n = 0, d = 0, nq = 0, dp = 0, mmax = 0;
  int wb = 1, W = 1, bw = 0;          // bits per attribute, field-packed words per row, bound words
  bool hig_log = false;               // HDPM_OPT_HIG_LOGSPACE (rmath.hpp log_hyperg_2F1)
  int Ws = 2;                         // words per bit-plane of the bit-sliced rows
  double gamma = 0;
  std::vector<int32_t> att;
  std::vector<double> v, w;
  std::vector<uint8_t> codes;  // row-major n x d
  DevBuf<uint8_t> d_codes_t;
  DevBuf<uint64_t> d_xpk;             // field-packed rows (tiled; histogram)
  DevBuf<uint64_t> d_xbs;             // bit-sliced rows (tiled; prepass)
  DevBuf<double> d_logn;
  std::vector<double> h_logn;
  // posterior analysis (hdpm_psm_*): label bytes, co-clustering counts, VI.lb sums
  DevBuf<int32_t> d_psm_trace, d_psm_cls;
  DevBuf<uint8_t> d_psm_lab;
  DevBuf<uint32_t> d_psm_cnt;
  DevBuf<double> d_psm_all, d_psm_same;
  int psm_N = 0, psm_M = 0;

  Rng rng;

  // internal_state.  Labels are device-authoritative after a sweep (host_c_valid).
  int K = 0;
  std::vector<int32_t> h_c;
  bool host_c_valid = false;
  bool host_c_device = false;         // h_c is a copy of the device labels (nothing to validate)
  std::vector<int32_t> h_counts;      // per label
  std::vector<uint8_t> h_center;      // K x d codes
  std::vector<double> h_sigma;        // K x d
  bool have_state = false;
  bool tables_dirty = true;
  uint64_t labels_version = 1;        // bumped whenever device labels may change
  uint64_t freq_version = 0;          // labels_version of the last full histogram (h_freq)
  bool stage_full = false;            // h_stage holds the tables of every label (last upload was full)

  DevBuf<int> d_c, d_counts, d_sol, d_los, d_src;
  DevBuf<uint8_t> d_slot_codes;
  DevBuf<double> d_slot_tab;
  DevBuf<uint64_t> d_slot_bnd;
  int scap = 0;
  bool last_fp = false;        // the last resolver launch was k_resolve_fp (diagnostics)
  int last_exact = 0;         // points the previous resolver launch decided one by one (block-mode choice)
  int last_listed = -1;       // points the previous launch's prepass listed (exact-rows grid), -1 unknown
  int last_fpg = 0;           // the previous launch's k_resolve_fpg grid (0: another resolver)
  double last_density = -1;   // ... per point of the range it covered (a restart covers the sweep's rest)
  bool last_unsettled = false;  // the previous launch exceeded its drift budget or restarted

  // latent pool
  int64_t P = 0;
  std::vector<uint8_t> h_pool_c;      // P x d codes (host-generated or user pools)
  std::vector<double> h_pool_s;       // P x d
  bool pool_on_device = false;        // device-generated: the parameters live in d_pool_*
  DevBuf<uint8_t> d_pool_codes;
  DevBuf<double> d_pool_tab;
  DevBuf<uint64_t> d_pool_bnd;
  DevBuf<uint64_t> d_pool_head;       // P x head_words (head_fits): the prepass's gather per latent pick
  int head_ha = 0, head_hb = 0;       // kernels.hpp "Pool-entry heads": h_a, h_b of this data
  DevBuf<double> d_pool_sig;          // P x d sigma (device generator)

  // pool-entry heads from the device tables and bound records (every pool install)
  void build_pool_heads() {
    if (!head_fits(wb, Ws) || P <= 0) return;
    d_pool_head.ensure((size_t)P * head_stride(wb, Ws));
    HIPCHK(launch_pool_heads(d_pool_tab.p, d_pool_bnd.p, P, d, wb, Ws, bw, head_ha, head_hb, d_pool_head.p, stream));
  }

  // stream-exact device pool generator (pool_gen.hpp)
  struct PoolGen {
    PoolPlan plan;
    bool planned = false;
    int G = 0, bpg = 0;               // jump tables for the slice generator
    DevBuf<uint64_t> jpoly;
    DevBuf<uint32_t> jidx;
    DevBuf<int> joff;
    DevBuf<uint32_t> init, raw;
    PinBuf<uint32_t> h_init, h_tail;
    DevBuf<uint64_t> bm;
    PinBuf<uint64_t> h_bm;
    DevBuf<int64_t> starts, cE, aux;
    DevBuf<uint32_t> T;
    DevBuf<int32_t> gj, gn, cidx;
    PinBuf<int64_t> h_starts;
    int64_t walk_fallbacks = 0;       // segment parses that left a window: serial host parse
    DevBuf<PoolClass> cls;
    DevBuf<int> runs;
    DevBuf<int32_t> att;
    DevBuf<uint64_t> gtab;
    DevBuf<int> err;
    PinBuf<int> h_err;
  } pg;

  // sweep scratch
  PinBuf<uint32_t> h_raw;
  DevBuf<uint32_t> d_raw;
  DevBuf<double> d_L;
  int Ecap = 0;
  DevBuf<double> d_margin;
  DevBuf<int> d_rowpos;
  DevBuf<int> d_list, d_cnt, d_dense, d_dense_total, d_spec, d_boff;
  DevBuf<double> d_spec_rad;
  DevBuf<int4> d_rq;
  DevBuf<uint64_t> d_csum;            // per-label cluster summary for the prepass
  DevBuf<unsigned> d_hist_part;
  DevBuf<long long> d_rprof;          // resolver phase times (debug mode bit 1)
  DevBuf<int> d_fpg;                   // k_resolve_fpg's cross-workgroup scratch
  DevBuf<int> d_wide_ctr;              // k_prepass_wide's chunk counter, k_exact_rows_mass's point counter
  DevBuf<int> d_warm;                  // zero gate word and scratch of warm_launch_kernels
  DevBuf<unsigned int> d_lmask;        // per exact row: latent columns holding head bounds
  bool kernels_warm = false;
  int fpg_grid_cache[65] = {0};        // its resident grid per resolver slot capacity (0: unknown, -1: none)
  int fpg_grid_m = -1;                 // ... for this m (the LDS of k_resolve_fpg depends on m)
  int& fpg_grid(int lcap, int m) {
    if (m != fpg_grid_m) {
      std::fill(fpg_grid_cache, fpg_grid_cache + 65, 0);
      fpg_grid_m = m;
    }
    return fpg_grid_cache[lcap];
  }
  PinBuf<int> h_ctl;                  // two blocks [ResolveCtl | pad to kCtlInts][resolver summary: 3 scap]
  // Consecutive sweeps alternate between the two control blocks (and resolver events), so a
  // sweep enqueued ahead (pre_enqueue) does not overwrite the one the host is reading.
  int par = 0;
  hipEvent_t ev_res[2] = {nullptr, nullptr};
  size_t ctl_stride() const { return kCtlInts + 3 * (size_t)scap; }
  ResolveCtl* ctl_at(int q) { return reinterpret_cast<ResolveCtl*>(h_ctl.p + (size_t)q * ctl_stride()); }
  // The next sweep enqueued before this iteration's update is joined (pre_enqueue): its
  // kernels wait on the device (k_pipe_wait) for the host's go (pipe_go) or abort
  // (pre_release); slots in host-coherent memory, gates on the device.
  PinBuf<PipeSlot> h_pipe;
  DevBuf<PipeGate> d_pipe;
  struct PreSweep {
    bool active = false;
    bool round_ok = false;             // round 0 was enqueued
    int par = 0, buf = -1, m = 0;
    bool track = false;
    bool dev = false;                  // its tables come from the device speculation (phd.stage)
    uint64_t gen[2] = {0, 0};          // window launches the kernels waited for
    std::chrono::steady_clock::time_point t_enq;   // the wait kernel was queued (pipe_go's deadline)
    bool au = false;                   // the wait kernel may give the go itself (PipeAuto)
  } pre;
  bool pipe_auto = true;               // device-side go for the device update's pipeline (HDPM_PIPE_AUTO=0: off)
  // PipeAuto: the wait kernel's decision (1: it gave the go, 2: it waits for the host), once it
  // has run (it runs once the previous sweep and the speculated update are done: microseconds)
  int pre_dev_decision() {
    if (!pre.active || !pre.au) return 0;
    const int* w = &h_pipe.p[pre.par].dev;
    const auto t0 = std::chrono::steady_clock::now();
    for (int polls = 0;; ++polls) {
      const int v = __atomic_load_n(w, __ATOMIC_ACQUIRE);
      if (v != 0) return v;
      HostPool::spin_pause();
      if ((polls & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
        // (the kernel behind the stream's work never ran: treat it as waiting for the flag)
        return 2;
      }
    }
  }
  // k_pipe_wait's limit in ticks of the 100 MHz clock (2 s), and whether pipe_go refuses a go
  // given after a quarter of it (HDPM_OPT_PIPE_WAIT_US; a negative value turns the check off, to
  // exercise the device-side gate-off and its recovery in neal8_sweep)
  long long pipe_limit_ticks = 200000000LL;
  bool pipe_host_check = true;
  // k_resolve_fpg's grid-barrier limit (ticks, 2 s) and the barrier at which workgroup 0 gives up
  // (testing, 0: none): HDPM_OPT_FPG_WAIT_US / HDPM_OPT_FPG_FAIL_AT.  A launch that gave up ends
  // as a restart and the next launch takes the one-workgroup resolver (fpg_skip).
  long long fpg_limit_ticks = 200000000LL;
  int fpg_fail_at = 0;
  bool fpg_skip = false;
  int last_xpath = 0;                  // the exact-rows kernel of the last launch (launch_exact_rows' path)
  int exact_pref = 0;                  // HDPM_OPT_EXACT_KERNEL (testing)
  double lat_negl = kLatNegligible;    // HDPM_OPT_LAT_NEGLIGIBLE (testing)
  long long sm_wide_ticks = 5000000;   // k_sm_scan_wide's barrier limit (100 MHz ticks; HDPM_OPT_SM_WIDE_WAIT_US)
  // restricted Gibbs samplers as one device chain (HDPM_OPT_SM_CHAIN: 0 off, the default -- the
  // chain's one-cluster device updates cost ~100 us each at C4 against ~45 us per cluster on the
  // host job, profiles/r06/sm_chain/ -- 1 on; >= 2 testing: the chain stops at step
  // sm_chain_mode - 2, split_merge.inl sm_chain; HDPM_SM_CHAIN=1 in the environment turns it on)
  int sm_chain_mode = [] {
    const char* e = std::getenv("HDPM_SM_CHAIN");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  bool deep_ok = false;                // set by iteration(): the next sweep may be enqueued ahead
  static constexpr size_t kCtlInts = 16;
  static_assert(sizeof(ResolveCtl) <= kCtlInts * sizeof(int), "control block");
  // cluster parameter upload staging (UploadLayout)
  // two pinned staging buffers: one can be filled (e.g. by the update_phi speculated for the
  // next sweep) while the last commit's copy from the other is still in flight
  PinBuf<uint8_t> h_stage_buf[3];
  hipEvent_t ev_stage_buf[3] = {nullptr, nullptr, nullptr};
  int stage_fill = 0, stage_last = 1;   // buffer being filled / last committed
  int stage_hold = -1;                  // filled by the speculative update_phi, not yet committed
  // the new tables of a full update_phi, committed after the next speculative update_phi is
  // started (flush_commit): buffer, entries
  // (dev: the speculative device update's tables, phd.stage)
  struct { bool active = false, dev = false; int buf = 0, nent = 0; } commit_later;
  DevBuf<uint8_t> d_stage;

  // statistics buffers.  d_freq holds freq[slot][j][level] and, while freq_dev_valid,
  // follows the labels through the sweeps incrementally (resolver move log); d_freq_m
  // takes masked (subset) histograms.
  DevBuf<unsigned> d_freq, d_freq2, d_freq_m;
  bool freq_dev_valid = false;
  // Debug bit 4 (value 16) recounts the tables for every update_phi instead of carrying them
  // through the sweep by the move log (the move log then does not run).  The carried tables
  // are used at every N: a sweep whose last point opened a cluster used to skip the sweep-end
  // kernels (kernels.hip sweep_done), which left the tables, and the labels, un-updated.
  bool recount_only() const { return (debug & 16) != 0; }
  uint64_t freq_d2h_version = 0;      // labels_version whose freq copy the sweep already started
  DevBuf<int> d_mlog, d_mcount;
  PinBuf<unsigned> h_freq;
  DevBuf<unsigned char> d_mask;
  PinBuf<unsigned char> h_mask;
  StreamAhead phi_stream;             // update_phi's slice of the R stream, generated ahead
  int64_t phi_prefetch = 4096;
  DevBuf<double> d_partial;
  PinBuf<double> h_partial;

  hdpm_stats stats{};
  int64_t launch_count = 0;           // resolver launches issued (prepass timing cadence)
  bool round_timed = false, round_fine = false;
  int64_t round_points = 0;
  // prepass timing of a sweep enqueued ahead (per control block: read one iteration later)
  bool pre_timed[2] = {false, false};
  hipEvent_t ev_pp[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  int debug = 0;
  // debug bit 1: per-iteration host timeline
  std::vector<std::pair<const char*, std::chrono::steady_clock::time_point>> trace;
  void mark(const char* what) {
    if (debug & 34) trace.emplace_back(what, std::chrono::steady_clock::now());
  }
  // debug bit 5: accumulate the per-iteration timeline (no extra synchronisation); printed
  // by the context's destructor
  std::vector<std::pair<std::string, double>> trace_sum;
  std::vector<std::vector<float>> trace_smp;   // per trace_sum entry: the samples (median / p90)
  void trace_add(const std::string& name, double us) {
    size_t q = 0;
    while (q < trace_sum.size() && trace_sum[q].first != name) ++q;
    if (q == trace_sum.size()) {
      trace_sum.emplace_back(name, 0.0);
      trace_smp.emplace_back();
    }
    trace_sum[q].second += us;
    trace_smp[q].push_back((float)us);
  }
  int64_t trace_iters = 0, trace_alloc0 = -1, trace_slow = 0;
  char spec_line[192] = {0};          // the last joined speculative update's stamps (debug bit 5)
  std::unordered_map<uint64_t, bool> beta_cache;

  SmWork sm;
  // scratch for host sampling
  std::vector<double> sp;
  std::vector<int> sperm;

  ~Ctx() {
    PoolScope scope(hpool);          // a speculative job still open is joined on this context's pool
    try {
      cancel_ahead();
    } catch (...) {
    }
    if (trace_iters > 0) {
      std::string line = "[timeline] us/iteration, mean [median p90]:";
      for (size_t q = 0; q < trace_sum.size(); ++q) {
        std::vector<float> v = trace_smp[q];
        std::sort(v.begin(), v.end());
        char buf[128];
        std::snprintf(buf, sizeof(buf), " %s %.1f [%.1f %.1f]", trace_sum[q].first.c_str(),
                      trace_sum[q].second / trace_iters, v.empty() ? 0.0 : v[v.size() / 2],
                      v.empty() ? 0.0 : v[v.size() * 9 / 10]);
        line += buf;
      }
      for (size_t q = 0; q < trace_sum.size(); ++q)
        if (trace_sum[q].first == "total") {
          line += "; totals in order:";
          for (size_t k = 0; k < trace_smp[q].size() && k < 40; ++k) {
            char buf[32];
            std::snprintf(buf, sizeof(buf), " %.0f", trace_smp[q][k]);
            line += buf;
          }
        }
      std::fprintf(stderr, "%s (%lld iterations, %lld device allocations after the first)\n", line.c_str(),
                   (long long)trace_iters, (long long)(g_dev_allocs.load() - trace_alloc0));
    }
    if (pstream) {
      (void)hipStreamSynchronize(pstream);
      if (dspec.ev) (void)hipEventDestroy(dspec.ev);
      if (dnext.ev) (void)hipEventDestroy(dnext.ev);
      if (ev_phd_free) (void)hipEventDestroy(ev_phd_free);
      if (phd.ev_last) (void)hipEventDestroy(phd.ev_last);
      (void)hipStreamDestroy(pstream);
    }
    if (cstream) {
      (void)hipStreamSynchronize(cstream);
      for (auto& sl : phis)
        if (sl.ev) (void)hipEventDestroy(sl.ev);
      (void)hipStreamDestroy(cstream);
    }
    if (gstream) {
      (void)hipStreamSynchronize(gstream);
      for (auto& w : win)
        if (w.done) (void)hipEventDestroy(w.done);
      if (pend.ev) (void)hipEventDestroy(pend.ev);
      (void)hipStreamDestroy(gstream);
    }
    if (stream) {
      (void)hipStreamSynchronize(stream);
      for (auto& e : ev) (void)hipEventDestroy(e);
      for (auto& e : ev_stage_buf)
        if (e) (void)hipEventDestroy(e);
      for (auto& e : ev_res)
        if (e) (void)hipEventDestroy(e);
      if (sm.ev_chain) (void)hipEventDestroy(sm.ev_chain);
      if (ev_labels) (void)hipEventDestroy(ev_labels);
      for (auto& pe : ev_pp)
        for (auto& e : pe)
          if (e) (void)hipEventDestroy(e);
      (void)hipStreamDestroy(stream);
    }
  }

  // ------------------------------------------------------------------ device random stream
  void rng_sync() {
    if (!pend.active) return;
    if (pend.from_raw) {
      HIPCHK(hipEventSynchronize(phidev.ev));
      mark("rs.slice");
      for (int i = 0; i < 624; ++i) rng.mt[i] = mt_untemper(pend.from_raw[i]);
    } else {
      HIPCHK(hipEventSynchronize(pend.ev));
      mark("rs.state");
      std::memcpy(rng.mt, pend.host_src ? pend.host_src : pend.arr.p, sizeof(rng.mt));
    }
    rng.mti = pend.mti;
    pend.active = false;
  }
  void rng_drop_pending() { pend.active = false; }

  void size_window(RngWindow& W, int64_t count, int64_t export_after) {
    const int head = W.mti0 >= 624 ? 0 : 624 - W.mti0;
    W.nblocks = count > head ? (int)((count - head + 623) / 624) : 0;
    W.count = count;
    // sized for any start offset (the block count varies with it), so a window of a given
    // length is never reallocated -- a free would synchronise the device
    // (with headroom: the span grows a little when the draws between sweeps do)
    if (W.raw.n < (size_t)count) W.raw.ensure((size_t)count + (size_t)count / 4);
    const size_t aw = (size_t)((count + 623) / 624 + 2) * 624;
    if (W.arrays.n < aw) W.arrays.ensure(aw + aw / 4);
    W.init.ensure(624);
    W.h_init.ensure(624);
    if (!W.done) HIPCHK(hipEventCreateWithFlags(&W.done, hipEventDisableTiming));
    // the host adopts states only at or after `export_after` draws into the window
    W.export_from = (int)std::max<int64_t>(1, (export_after - head) / 624 - 1);
    W.export_after = export_after;
  }
  // a generator launch may overwrite buffers the copy stream still reads
  void gstream_after_copies() {
    if (pend.ev) HIPCHK(hipStreamWaitEvent(gstream, pend.ev, 0));
    for (auto& sl : phis)
      if (sl.ev) HIPCHK(hipStreamWaitEvent(gstream, sl.ev, 0));
  }
  void run_window(RngWindow& W) {
    ensure_jump(W.count);
    const bool multi = mt_G > 1 && W.count >= (int64_t)mt_G * 624 * 8;
    MtGenArgs a{W.init_src ? W.init_src : W.init.p, W.mti0, W.count, W.raw.p, W.arrays.p, W.nblocks, W.export_from,
                multi ? d_jpoly.p : nullptr, d_jidx.p, d_joff.p, mt_bpg, multi ? mt_G : 1};
    HIPCHK(launch_mt_gen(a, gstream));
    HIPCHK(hipEventRecord(W.done, gstream));
    W.gen++;
    stats.rng_windows++;
    W.valid = true;
  }

  // Window starting at the host stream's current state.
  void launch_window(RngWindow& W, int64_t count, int64_t export_after = 0) {
    rng_sync();
    if (rng.mti == 625) {  // never seeded: R seeds with 4357 (MT_sgenrand) on the first draw
      uint32_t seed = 4357;
      for (int i = 0; i < 624; i++) {
        rng.mt[i] = seed & 0xffff0000u;
        seed = 69069u * seed + 1u;
        rng.mt[i] |= (seed & 0xffff0000u) >> 16;
        seed = 69069u * seed + 1u;
      }
      rng.mti = 624;
    }
    HIPCHK(hipStreamSynchronize(gstream));  // previous use of W's buffers is complete
    if (cstream) HIPCHK(hipStreamSynchronize(cstream));
    W.mti0 = rng.mti;
    W.start_pos = rng.pos;
    W.epoch = rng.epoch;
    size_window(W, count, export_after);
    // the other window's buffers too, now: its first launch comes mid-chain, where an
    // allocation would stall the iteration
    RngWindow& O = (&W == &win[0]) ? win[1] : win[0];
    if (O.raw.n < W.raw.n) O.raw.ensure(W.raw.n);
    if (O.arrays.n < W.arrays.n) O.arrays.ensure(W.arrays.n);
    O.init.ensure(624);
    O.h_init.ensure(624);
    if (!O.done) HIPCHK(hipEventCreateWithFlags(&O.done, hipEventDisableTiming));
    std::memcpy(W.h_init.p, rng.mt, sizeof(rng.mt));
    HIPCHK(hipMemcpyAsync(W.init.p, W.h_init.p, 624 * 4, hipMemcpyHostToDevice, gstream));
    W.init_src = W.init.p;
    run_window(W);
  }

  // Block and mti of the state after `target` draws, inside window W (R keeps mti = 624
  // at a block edge).  blk 0 = W's initial array.
  void locate(const RngWindow& W, uint64_t target, int64_t* blk, int* mti) const {
    const uint64_t r = target - W.start_pos;
    const uint64_t head = W.mti0 >= 624 ? 0 : 624 - W.mti0;
    if (r < head) {
      *blk = 0;
      *mti = W.mti0 + (int)r;
      return;
    }
    const uint64_t b = 1 + (r - head) / 624, k = (r - head) % 624;
    *blk = (int64_t)(k == 0 ? b - 1 : b);
    *mti = k == 0 ? 624 : (int)k;
    if (*blk != 0 && *blk < W.export_from) throw HipError{hipErrorInvalidValue, "rng window export"};
  }

  // Window Wn starting at position `target` of window Ws, initialised on the device from
  // Ws's exported arrays (no host round trip).
  void launch_window_from(RngWindow& Wn, RngWindow& Ws, uint64_t target, int64_t count, int64_t export_after) {
    int64_t blk;
    int mti;
    locate(Ws, target, &blk, &mti);
    Wn.mti0 = mti;
    Wn.start_pos = target;
    Wn.epoch = rng.epoch;
    gstream_after_copies();
    size_window(Wn, count, export_after);
    if (blk == 0) {
      // inside Ws's initial array, which may live in Wn's own exports: copy it out first
      HIPCHK(hipMemcpyAsync(Wn.init.p, Ws.init_src ? Ws.init_src : Ws.init.p, 624 * 4, hipMemcpyDeviceToDevice,
                            gstream));
      Wn.init_src = Wn.init.p;
    } else {
      // read in place: Ws's exports are rewritten only by a later launch on this stream
      Wn.init_src = Ws.arrays.p + (blk - 1) * 624;
    }
    HIPCHK(hipMemcpyAsync(Wn.h_init.p, Wn.init_src, 624 * 4, hipMemcpyDeviceToHost, gstream));
    run_window(Wn);
  }

  // Jump polynomials z^(624 * bpg * g) mod phi for g < G, built once per window size class
  // and checked on the host against direct twisting.
  void ensure_jump(int64_t count) {
    static const int G = [] {
      const char* e = std::getenv("HDPM_MT_WORKGROUPS");
      const int g = e ? std::atoi(e) : 0;
      return g >= 2 && g <= 4096 ? g : 256;
    }();
    if (count < (int64_t)G * 624 * 8) return;
    if (mt_G == G && count <= (int64_t)624 * G * mt_bpg) return;
    // headroom so later, slightly larger windows (sweep + draws between sweeps) reuse it
    const int bpg = (int)((count * 5 / 4 + 624 * G - 1) / (624 * G));
    HIPCHK(hipStreamSynchronize(gstream));   // no generator may still read the tables
    if (!build_jump(d_jpoly, d_jidx, d_joff, G, bpg)) return;
    mt_G = G;
    mt_bpg = bpg;
  }

  // Tables of z^(624 bpg g - 1) mod phi, g = 1..G-1 (set-bit lists for the generator's
  // correlation), the chain split over host threads (one exponentiation per thread, then
  // multiplications by z^(624 bpg)); checked against direct twisting for segments 1 and 2
  // (and G/2, G-1 when that is cheap).
  bool build_jump(DevBuf<uint64_t>& jpoly, DevBuf<uint32_t>& jidx, DevBuf<int>& joff, int G, int bpg) {
    static const Poly phi = mt_charpoly();
    if (phi.empty()) return false;
    const uint64_t J = (uint64_t)624 * bpg;
    const Poly pj = poly_xpow(J, phi);
    std::vector<uint64_t> all((size_t)G * 312, 0);
    const int T = std::max(1, std::min(host_threads(), (G - 1) / 8));
    const int per = (G - 1 + T - 1) / T;
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) {
      const int g0 = 1 + t * per, g1 = std::min(G, g0 + per);
      if (g0 >= g1) break;
      th.emplace_back([&, g0, g1] {
        Poly p = poly_xpow(J * g0 - 1, phi);
        for (int g = g0; g < g1; ++g) {
          std::memcpy(&all[(size_t)g * 312], p.data(), 312 * 8);
          if (g + 1 < g1) p = poly_mulmod(p, pj, phi);
        }
      });
    }
    for (auto& x : th) x.join();
    {
      Rng r;
      r.set_seed(20241015u);
      (void)r.raw();
      Rng q = r;
      int64_t done = 0;
      std::vector<int> segs{1, std::min(2, G - 1)};
      if ((int64_t)(G - 1) * bpg <= 20000) segs.insert(segs.end(), {G / 2, G - 1});
      std::sort(segs.begin(), segs.end());
      for (int g : segs) {
        uint32_t jumped[624];
        Poly pg(all.begin() + (size_t)g * 312, all.begin() + (size_t)(g + 1) * 312);
        mt_jump_host(r.mt, pg, jumped);
        for (; done < (int64_t)g * bpg; ++done) q.twist();
        if (std::memcmp(jumped, q.mt, sizeof(jumped)) != 0) return false;
      }
    }
    std::vector<int> off(G + 1, 0);
    std::vector<uint32_t> idx;
    for (int g = 0; g < G; ++g) {
      off[g] = (int)idx.size();
      if (g > 0)
        for (int i = 0; i < kMtDeg; ++i)
          if ((all[(size_t)g * 312 + (i >> 6)] >> (i & 63)) & 1u) idx.push_back((uint32_t)i);
    }
    off[G] = (int)idx.size();
    jpoly.ensure(all.size());
    HIPCHK(hipMemcpy(jpoly.p, all.data(), all.size() * 8, hipMemcpyHostToDevice));
    jidx.ensure(std::max<size_t>(idx.size(), 1));
    HIPCHK(hipMemcpy(jidx.p, idx.data(), idx.size() * 4, hipMemcpyHostToDevice));
    joff.ensure(off.size());
    HIPCHK(hipMemcpy(joff.p, off.data(), off.size() * 4, hipMemcpyHostToDevice));
    return true;
  }

  bool covers(const RngWindow& W, uint64_t p, int64_t n) const {
    return W.valid && W.epoch == rng.epoch && W.start_pos <= p && p + n <= W.start_pos + (uint64_t)W.count &&
           p + n >= W.start_pos + (uint64_t)W.export_after;
  }

  // The index (1..624; 0: none) of position p in its block of the stream (the same block edges
  // in every window)
  static int mti_at(const RngWindow& W, uint64_t p) {
    if (p < W.start_pos) return 0;
    const uint64_t r = p - W.start_pos;
    const uint64_t head = W.mti0 >= 624 ? 0 : 624 - W.mti0;
    if (r < head) return W.mti0 + (int)r;
    const uint64_t k = (r - head) % 624;
    return k == 0 ? 624 : (int)k;
  }
  // an update's stream slice: from position rng.pos in window W
  void phi_raw(PhiArgs& a, const RngWindow& W) const {
    a.raw = W.raw.p + (rng.pos - W.start_pos);
    a.nraw = (int64_t)(W.start_pos + (uint64_t)W.count - rng.pos);
    a.raw_back = (int64_t)(rng.pos - W.start_pos);
    a.mti_pos = mti_at(W, rng.pos);
    a.pos0 = (int64_t)rng.pos;
  }
  // After a device update that consumed up to `target`: the state the fast path copied out
  // (`state`: the block's 624 words, then its index; k_phi2_values), else adopt_state_at.
  void adopt_after_phi(RngWindow& W, uint64_t target, const uint32_t* state) {
    if (state) {
      const int mt = (int)state[624];
      if (mt >= 1 && mt <= 624 && mt == mti_at(W, target)) {
        for (int i = 0; i < 624; ++i) rng.mt[i] = mt_untemper(state[i]);
        rng.mti = mt;
        pend.active = false;
        rng.pos = target;
        stats.phi_state_direct++;
        return;
      }
    }
    adopt_state_at(W, target);
  }

  // Make the host stream continue at position `target` inside window W: rng.pos now, the
  // state array asynchronously (rng_sync()).
  void adopt_state_at(RngWindow& W, uint64_t target) {
    int64_t blk;
    int mti;
    locate(W, target, &blk, &mti);
    if (!pend.ev) HIPCHK(hipEventCreateWithFlags(&pend.ev, hipEventDisableTiming));
    HIPCHK(hipStreamWaitEvent(cstream, W.done, 0));
    if (blk == 0) {
      pend.host_src = W.h_init.p;     // valid once W's init has landed (W.done)
    } else {
      pend.arr.ensure(624);
      pend.host_src = nullptr;
      HIPCHK(hipMemcpyAsync(pend.arr.p, W.arrays.p + (blk - 1) * 624, 624 * 4, hipMemcpyDeviceToHost, cstream));
    }
    HIPCHK(hipEventRecord(pend.ev, cstream));
    pend.mti = mti;
    pend.from_raw = nullptr;
    pend.active = true;
    rng.pos = target;
  }

  // update_phi's slice [target, target + N) with the state arrays of its twists, copied from
  // window W when it holds them (else the host generates the slice itself).
  // One copy serves both: the words of the state's block from its start (the state after
  // `target` draws is that block untempered, rng_sync) through the block of the slice's
  // last word.  False when window W does not hold them (then adopt_state_at).
  bool phi_device_prefetch(const RngWindow& W, uint64_t target, int64_t N) {
    phidev.valid = false;
    // the state's position in its block (one stream: the same block edges in every window)
    const int mti = mti_at(W, target);
    // (a block that starts before the stream's first word: no window holds it)
    if (mti < 1 || target < (uint64_t)mti) return false;
    const uint64_t s_blk = target - (uint64_t)mti;              // first word of the state's block
    const int64_t words = 624 * ((mti + N - 1) / 624 + 1);       // through the block of word N - 1
    PhiSlice* hit = nullptr;
    for (auto& sl : phis)
      if (sl.valid && sl.epoch == rng.epoch && sl.s0 <= s_blk && s_blk - sl.s0 + (uint64_t)words <= (uint64_t)sl.words)
        hit = &sl;
    if (hit) {
      stats.phi_lookahead_hits++;
    } else {
      // from whichever window holds the whole slice (one that ends inside it is followed by
      // the next, which starts earlier)
      const RngWindow* X = nullptr;
      for (const auto& w : win)
        if (w.valid && w.epoch == rng.epoch && s_blk >= w.start_pos &&
            s_blk - w.start_pos + (uint64_t)words <= (uint64_t)w.count && (!X || w.start_pos < X->start_pos))
          X = &w;                         // the earlier window: generated first
      if (!X) return false;
      hit = phi_slice_copy(*X, s_blk, words, nullptr);
    }
    hit->stamp = ++phis_clock;
    phidev.valid = true;
    phidev.pos = target;
    phidev.epoch = rng.epoch;
    phidev.mti = mti;
    phidev.N = N;
    phidev.ev = hit->ev;
    phidev.blk = hit->buf.p + (s_blk - hit->s0);
    // the host stream continues at target: its state arrives with the copy
    pend.active = true;
    pend.from_raw = phidev.blk;
    pend.mti = mti;
    rng.pos = target;
    return true;
  }
  // Words [s0, s0 + words) of window W into the least recently used ring slot other than
  // `keep` (asynchronous, on the copy stream).
  PhiSlice* phi_slice_copy(const RngWindow& W, uint64_t s0, int64_t words, const PhiSlice* keep) {
    PhiSlice* sl = nullptr;
    for (auto& c : phis)
      if (&c != keep && (!sl || c.stamp < sl->stamp)) sl = &c;
    // with headroom: a pinned reallocation (hipHostFree) would synchronise the device
    if (sl->buf.n < (size_t)words) {
      if (sl->ev) HIPCHK(hipEventSynchronize(sl->ev));
      sl->buf.ensure(std::max<size_t>(2 * (size_t)words, 1 << 15));
    }
    if (!sl->ev) HIPCHK(hipEventCreateWithFlags(&sl->ev, hipEventDisableTiming));
    HIPCHK(hipStreamWaitEvent(cstream, W.done, 0));
    HIPCHK(hipMemcpyAsync(sl->buf.p, W.raw.p + (s0 - W.start_pos), (size_t)words * 4, hipMemcpyDeviceToHost, cstream));
    HIPCHK(hipEventRecord(sl->ev, cstream));
    sl->valid = true;
    sl->s0 = s0;
    sl->words = words;
    sl->epoch = rng.epoch;
    sl->stamp = ++phis_clock;
    return sl;
  }
  // The stretch device_draws noted for the next update's slice (the draws of the next sweep
  // after at most a slice's worth of this update's), copied now: off the iteration's
  // critical path, and landed by the time the next sweep's draws are reserved.
  void phi_lookahead() {
    if (!look_from || (debug & 1048576)) return;
    const uint64_t from = look_from;
    look_from = 0;
    for (auto& sl : phis)
      if (sl.valid && sl.epoch == rng.epoch && sl.s0 <= from && from + (uint64_t)look_words <= sl.s0 + (uint64_t)sl.words)
        return;
    const RngWindow* X = nullptr;
    for (auto& W : win)
      if (W.valid && W.epoch == rng.epoch && W.start_pos <= from &&
          from + (uint64_t)look_words <= W.start_pos + (uint64_t)W.count && (!X || W.start_pos < X->start_pos))
        X = &W;
    // a window still being generated would hold the in-order copy stream behind it
    if (X && hipEventQuery(X->done) == hipSuccess) {
      const RngWindow& W = *X;
      {
        const PhiSlice* keep = nullptr;
        for (auto& sl : phis)
          if (phidev.valid && sl.valid && phidev.blk >= sl.buf.p && phidev.blk < sl.buf.p + sl.words) keep = &sl;
        (void)phi_slice_copy(W, from, look_words, keep);
        stats.phi_lookahead_copies++;
      }
    }
  }

  // Device pointer to the next n raw draws of the stream; advances the host stream past
  // them and starts generating the following window from where they end.
  //
  // Windows span many sweeps (`window_span`): one jump-ahead + twist launch serves ~16
  // sweeps and the draws between them, instead of one launch (dominated by the jump) per
  // sweep.  The next window is launched from the end of the current sweep's draws when the
  // current one has fewer than `kLead` sweeps' worth left, so it is ready well before use.
  // (a window takes ~0.5 ms to generate at C5, several sweeps' time: started 8 sweeps
  // ahead, it is done before the first draw from it)
  static constexpr int kLead = 8;
  int64_t window_span(int64_t n) const {
    // independent of cmax unless the draws between sweeps outgrow its allowance, so the
    // span (window buffers, jump tables) stays fixed
    const int64_t cap = (int64_t)1 << 27;      // 512 MB of draws (+ 512 MB of exported arrays)
    return std::max(n + cmax, std::min<int64_t>(16 * (n + (1 << 18)), cap));
  }
  const uint32_t* device_draws(int64_t n) {
    RngWindow* W = nullptr;
    for (auto& w : win)
      if (covers(w, rng.pos, n) && (!W || w.start_pos < W->start_pos)) W = &w;
    if (!W) {
      if (win[0].valid || win[1].valid) cmax = std::min<int64_t>(cmax * 2, 1 << 26);
      W = &win[0];
      launch_window(*W, window_span(n), n);
      stats.rng_windows_fresh++;
    }
    mark("dd.window");
    HIPCHK(hipStreamWaitEvent(stream, W->done, 0));
    const uint32_t* p = W->raw.p + (rng.pos - W->start_pos);
    const uint64_t target = rng.pos + n;
    if (!phi_device_prefetch(*W, target, phi_prefetch)) adopt_state_at(*W, target);
    mark("dd.state");
    // the next sweep's update slice starts after this update's draws (at most about a
    // slice) and the next sweep's n: fetched ahead by phi_lookahead
    look_from = target + (uint64_t)n > 624 ? target + (uint64_t)n - 624 : 0;
    look_words = 2 * phi_prefetch + 3 * 624;
    RngWindow* other = (W == &win[0]) ? &win[1] : &win[0];
    const bool ahead = other->valid && other->epoch == rng.epoch && other->start_pos > W->start_pos;
    const uint64_t wend = W->start_pos + (uint64_t)W->count;
    if (!ahead && wend < target + (uint64_t)(kLead * (n + cmax)))
      launch_window_from(*other, *W, target, window_span(n), n);
    return p;
  }

  // ------------------------------------------------------------------ helpers
  void tables_for(const uint8_t* cen, const double* sig, uint8_t* out_codes, double* out_tab) const {
    std::memset(out_codes, 0, dp);
    for (int j = 0; j < d; ++j) {
      out_codes[j] = cen[j];
      dhamming_pair(sig[j], att[j], &out_tab[2 * j], &out_tab[2 * j + 1]);
    }
  }

  // Bound data of one parameter entry (kernels.hpp, "Bound data per parameter entry").
  void bounds_for(const uint8_t* cen, const double* tab, uint64_t* out) const {
    std::memset(out, 0, (size_t)bw * 8);
    long double A = 0.0L, sc = 0.0L;
    double dmax = 0.0, dmin = INFINITY;
    for (int j = 0; j < d; ++j) {
      const unsigned code = cen[j] - 1u;
      for (int b = 0; b < wb; ++b)
        if ((code >> b) & 1u) out[b * Ws + (j >> 6)] |= 1ull << (j & 63);
      A += (long double)tab[2 * j];
      sc += (long double)std::max(std::fabs(tab[2 * j]), std::fabs(tab[2 * j + 1]));
      const double dj = tab[2 * j] - tab[2 * j + 1];
      dmax = std::max(dmax, dj);
      dmin = std::min(dmin, dj);
    }
    const double delta = dmax > 0 ? dmax / ((1 << kQ) - 1) : 0.0;
    for (int j = 0; j < d; ++j) {
      const double dj = tab[2 * j] - tab[2 * j + 1];
      int q = delta > 0 ? (int)std::floor(dj / delta) : 0;
      q = std::min(std::max(q, 0), (1 << kQ) - 1);
      while (q > 0 && delta * q > dj) --q;
      while (q < (1 << kQ) - 1 && delta * (q + 1) <= dj) ++q;
      for (int b = 0; b < kQ; ++b)
        if ((q >> b) & 1) out[(wb + b) * Ws + (j >> 6)] |= 1ull << (j & 63);
    }
    double* s = reinterpret_cast<double*>(out + (wb + kQ) * Ws);
    s[0] = (double)A;
    s[1] = delta;
    s[2] = dmin > 0 ? dmin : 0.0;
    s[3] = (double)sc;
  }

  void ensure_slots(int need) {
    if (need <= scap) return;
    int nc = std::max(need, std::max(2 * scap, 64));
    d_counts.ensure(nc, true, stream);
    d_sol.ensure(nc, true, stream);
    d_los.ensure(nc, true, stream);
    d_src.ensure(nc, true, stream);
    d_slot_codes.ensure((size_t)nc * dp, true, stream);
    d_slot_tab.ensure((size_t)nc * 2 * d, true, stream);
    d_slot_bnd.ensure((size_t)nc * bw, true, stream);
    d_freq.ensure((size_t)nc * d * mmax, true, stream);
    d_freq2.ensure((size_t)nc * d * mmax);
    scap = nc;
  }

  // Cluster parameters of `which` (nullptr: labels 0..K-1 with counts and identity slot
  // maps) through the pinned staging buffer: one copy + one scatter kernel, no host wait.
  // Three steps so that callers can fill entries concurrently: stage_begin (wait until
  // the previous upload has left the buffer), stage_entry per entry r (label k),
  // stage_commit (copy + scatter).
  UploadLayout stage_begin(int nent) {
    const UploadLayout L = upload_layout(nent, dp, d, bw);
    auto pick = [&] {
      int f = 0;
      while (f < 3 && (f == stage_last || f == stage_hold || (commit_later.active && f == commit_later.buf))) ++f;
      return f;
    };
    int f = pick();
    if (f >= 3) {                                   // a commit deferred and another update held
      flush_commit();
      f = pick();
    }
    stage_fill = f;
    hipEvent_t& ev = ev_stage_buf[stage_fill];
    if (!ev) HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIPCHK(hipEventSynchronize(ev));                // the upload before last has left this buffer
    PinBuf<uint8_t>& hb = h_stage_buf[stage_fill];
    // coherent: a sweep enqueued ahead scatters from it in place (pre_enqueue)
    if (hb.n < L.bytes) hb.ensure(L.bytes + L.bytes / 2 + 4096, hipHostMallocCoherent);
    d_stage.ensure(L.bytes);
    return L;
  }
  uint8_t* stage_ptr() { return h_stage_buf[stage_fill].p; }
  void stage_entry(const UploadLayout& L, int r, int k) {
    uint8_t* st = stage_ptr();
    double* tt = (double*)(st + L.off_tab) + (size_t)r * 2 * d;
    tables_for(&h_center[(size_t)k * d], &h_sigma[(size_t)k * d], st + L.off_codes + (size_t)r * dp, tt);
    bounds_for(&h_center[(size_t)k * d], tt, (uint64_t*)(st + L.off_bnd) + (size_t)r * bw);
    ((int*)(st + L.off_counts))[r] = h_counts[k];
    ((int*)(st + L.off_slot))[r] = k;
  }
  void stage_commit(const UploadLayout& L, int nent, bool full) {
    if (stage_hold == stage_fill) stage_hold = -1;
    HIPCHK(hipMemcpyAsync(d_stage.p, stage_ptr(), L.bytes, hipMemcpyHostToDevice, stream));
    HIPCHK(hipEventRecord(ev_stage_buf[stage_fill], stream));
    stage_last = stage_fill;
    stage_full = full;
    HIPCHK(launch_scatter_clusters(d_stage.p, nent, dp, d, bw, full ? 1 : 0, d_slot_codes.p, d_slot_tab.p,
                                   d_slot_bnd.p, d_counts.p, d_sol.p, d_los.p, d_src.p, stream));
  }

  bool defer_commit = false;           // set by iteration() around its update_phi
  void flush_commit() {
    if (!commit_later.active) return;
    commit_later.active = false;
    if (commit_later.dev) {
      commit_later.dev = false;
      scatter_dev_stage(commit_later.nent);
      return;
    }
    stage_fill = commit_later.buf;
    stage_commit(upload_layout(commit_later.nent, dp, d, bw), commit_later.nent, true);
  }

  void stage_upload(const std::vector<int>* which) {
    const int nent = which ? (int)which->size() : K;
    if (nent == 0) return;
    const UploadLayout L = stage_begin(nent);
    pool_for(nent, [&](int r) { stage_entry(L, r, which ? (*which)[r] : r); });
    stage_commit(L, nent, which == nullptr);
  }

  // Upload label tables, counts and identity slot maps for labels 0..K-1.
  void upload_clusters() {
    ensure_slots(K + 2);
    stage_upload(nullptr);
    tables_dirty = false;
  }

  // Upload tables of the labels in `which` only (after update_phi on a subset).
  void upload_some(const std::vector<int>& which) { stage_upload(&which); }

  // moves of the last sweep to apply to the host mirror from the move log (see neal8_sweep)
  int mirror_moves = 0;
  // hdpm_iterations_record's centers / sigmas of the saved iterations (K x d rows each)
  std::vector<uint8_t> rec_cen;
  std::vector<double> rec_sig;
  void record_params() {
    rec_cen.insert(rec_cen.end(), h_center.begin(), h_center.begin() + (size_t)K * d);
    rec_sig.insert(rec_sig.end(), h_sigma.begin(), h_sigma.begin() + (size_t)K * d);
  }
  // The labels on the host before the device can change them again (the recording path, right
  // after a sweep): the mirror, the move log applied to it, or a download (on cstream: the
  // sweep stream may hold a sweep enqueued ahead behind its wait kernel).
  void capture_labels() {
    if (host_c_valid) return;
    // behind the last sweep end (slot ids -> labels, the move log complete); a sweep enqueued
    // ahead sits behind it on `stream`, so the wait cannot reach that sweep's gate
    if (ev_labels) HIPCHK(hipStreamWaitEvent(cstream, ev_labels, 0));
    if (mirror_moves > 0) {
      mlog_h.resize((size_t)3 * mirror_moves);
      HIPCHK(hipMemcpyAsync(mlog_h.data(), d_mlog.p, mlog_h.size() * 4, hipMemcpyDeviceToHost, cstream));
      HIPCHK(hipStreamSynchronize(cstream));
      for (int q = 0; q < mirror_moves; ++q) h_c[mlog_h[3 * q]] = mlog_h[3 * q + 2];
      mirror_moves = 0;
      host_c_valid = true;
      host_c_device = true;
      stats.labels_mirrored++;
      return;
    }
    h_c.resize(n);
    HIPCHK(hipMemcpyAsync(h_c.data(), d_c.p, (size_t)n * 4, hipMemcpyDeviceToHost, cstream));
    HIPCHK(hipStreamSynchronize(cstream));
    host_c_valid = true;
    host_c_device = true;
    stats.labels_downloaded++;
  }
  std::vector<int> mlog_h;

  void download_labels() {
    if (host_c_valid) return;
    h_c.resize(n);
    HIPCHK(hipMemcpyAsync(h_c.data(), d_c.p, (size_t)n * 4, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    host_c_valid = true;
    host_c_device = true;
  }

  void upload_labels() {
    d_c.ensure(n);
    HIPCHK(hipMemcpyAsync(d_c.p, h_c.data(), (size_t)n * 4, hipMemcpyHostToDevice, stream));
    labels_version++;
    freq_dev_valid = false;
    HIPCHK(hipStreamSynchronize(stream));
    host_c_valid = true;
    host_c_device = false;
  }

  void recount() {
    h_counts.assign(K, 0);
    for (int i = 0; i < n; ++i)
      if (h_c[i] >= 0 && h_c[i] < K) h_counts[h_c[i]]++;
  }

  bool beta_path(double vv, double ww, double mj) {
    uint64_t key;
    {
      uint64_t a, b, c;
      std::memcpy(&a, &vv, 8);
      std::memcpy(&b, &ww, 8);
      std::memcpy(&c, &mj, 8);
      key = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full ^ c;
    }
    auto it = beta_cache.find(key);
    if (it != beta_cache.end()) return it->second;
    bool r = rhig_beta_path(vv, ww, mj);
    if (beta_cache.size() < (1u << 20)) beta_cache.emplace(key, r);
    return r;
  }

  // sample_sigma_1_cluster (cf:218-235)
  int sample_sigma(const double* vv, const double* ww, double* out) {
    rng_sync();
    for (int j = 0; j < d; ++j) {
      int e = kOk;
      const double mj = (double)att[j];
      out[j] = rhig1_decided(rng, vv[j], ww[j], mj, beta_path(vv[j], ww[j], mj), &e, hig_log);
      if (e) return e;
    }
    return kOk;
  }
  // sample_sigma with the per-attribute branch tests (hg:359, the qbeta) and rbeta constants
  // evaluated on the host pool first; the draws stay in attribute order on this thread, so
  // the stream and the values are sample_sigma's.  For wide rows (split-merge at large D).
  int sample_sigma_wide(const double* vv, const double* ww, double* out) {
    if (d < 128) return sample_sigma(vv, ww, out);
    rng_sync();
    std::vector<char> bp(d);
    std::vector<RBeta> setup(d);
    pool_for(d, [&](int j) {
      const double mj = (double)att[j];
      bp[j] = rhig_beta_path(vv[j], ww[j], mj);
      if (bp[j]) setup[j] = rbeta_setup(ww[j] + 1, vv[j] - 1);
    }, 16);
    for (int j = 0; j < d; ++j) {
      const double m = (double)att[j];
      double u;
      if (bp[j]) {                                   // hg:359-366
        double x = rbeta_draw(rng, setup[j]);
        while (x > (m - 1) / m) x = rbeta_draw(rng, setup[j]);
        u = x / ((m - 1) * (1 - x));
      } else {                                       // hg:367-371
        int e = kOk;
        const double Omega = rng.unif();
        u = bisec_hyper2(ww[j], vv[j], m, Omega, &e, hig_log);
        if (e) return e;
      }
      out[j] = -1 / std::log(u);
    }
    return kOk;
  }
  // sample_center_1_cluster without probabilities (cf:198-199)
  void sample_center_uniform(uint8_t* out) {
    rng_sync();
    for (int j = 0; j < d; ++j) out[j] = (uint8_t)(int)(att[j] * rng.unif() + 1);
  }

  // ------------------------------------------------------------------ data
  int set_data(const uint8_t* x, int n_, int d_, const int32_t* attr, double g, const double* vv,
               const double* ww) {
    if (n_ <= 0 || d_ <= 0) { err = "n and d must be positive"; return kArg; }
    for (int j = 0; j < d_; ++j)
      if (attr[j] < 1 || attr[j] > 255) { err = "attrisize must be in 1..255"; return kArg; }
    for (int64_t i = 0; i < (int64_t)n_ * d_; ++i) {
      const int j = (int)(i % d_);
      if (x[i] < 1 || x[i] > attr[j]) { err = "codes must lie in 1..attrisize[j]"; return kArg; }
    }
    n = n_; d = d_; nq = (d + 15) / 16; dp = nq * 16; gamma = g;
    pg.planned = false;
    phd.ready = false;
    dev_ll_version = 0;
    att.assign(attr, attr + d);
    v.assign(vv, vv + d);
    w.assign(ww, ww + d);
    mmax = *std::max_element(att.begin(), att.end());
    codes.assign(x, x + (size_t)n * d);
    const int64_t n64 = ((int64_t)n + 63) / 64 * 64;
    std::vector<uint8_t> t((size_t)n64 * dp, 0);
    for (int64_t i = 0; i < n; ++i)
      for (int j = 0; j < d; ++j) t[tiled_offset(i, j, nq)] = codes[(size_t)i * d + j];
    d_codes_t.ensure(t.size());
    HIPCHK(hipMemcpyAsync(d_codes_t.p, t.data(), t.size(), hipMemcpyHostToDevice, stream));
    // packed rows: code-1 in wb bits (wb = smallest power of two with 2^wb >= mmax)
    wb = mmax <= 2 ? 1 : mmax <= 4 ? 2 : mmax <= 16 ? 4 : 8;
    const int F = 64 / wb;
    W = (d + F - 1) / F;
    std::vector<uint64_t> xp((size_t)n64 * W, 0);
    for (int64_t i = 0; i < n; ++i)
      for (int j = 0; j < d; ++j)
        xp[packed_offset(i, j / F, W)] |= (uint64_t)(codes[(size_t)i * d + j] - 1) << ((j % F) * wb);
    d_xpk.ensure(xp.size());
    HIPCHK(hipMemcpyAsync(d_xpk.p, xp.data(), xp.size() * 8, hipMemcpyHostToDevice, stream));
    // bit-sliced rows (kernels.hpp)
    Ws = plane_words(d);
    bw = bound_words(wb, Ws);
    {
      // mismatches of a point with a uniform latent center: mean and sd over the attributes
      double mu = 0.0, s2 = 0.0;
      for (int j = 0; j < d; ++j) {
        const double q = 1.0 / att[j];
        mu += 1.0 - q;
        s2 += (1.0 - q) * q;
      }
      head_ha = std::max(0, (int)std::floor(mu - 4.0 * std::sqrt(s2)));
      head_hb = std::max(0, (int)std::floor(mu - 1.25 * std::sqrt(s2)));
    }
    {
      const int Wr = wb * Ws;
      std::vector<uint64_t> xs((size_t)n64 * Wr, 0);
      parallel_for(n, [&](int64_t a0, int64_t a1) {
        for (int64_t i = a0; i < a1; ++i)
          for (int j = 0; j < d; ++j) {
            const unsigned code = codes[(size_t)i * d + j] - 1u;
            for (int b = 0; b < wb; ++b)
              if ((code >> b) & 1u) xs[packed_offset(i, b * Ws + (j >> 6), Wr)] |= 1ull << (j & 63);
          }
      });
      d_xbs.ensure(xs.size());
      HIPCHK(hipMemcpyAsync(d_xbs.p, xs.data(), xs.size() * 8, hipMemcpyHostToDevice, stream));
    }
    HIPCHK(hipStreamSynchronize(stream));
    scap = 0;   // slot arrays are re-laid out for the new bound size on next use
    freq_dev_valid = false;
    d_slot_bnd.release();
    h_logn.resize((size_t)n + 2);
    h_logn[0] = -INFINITY;
    for (int k = 1; k < n + 2; ++k) h_logn[k] = std::log((double)k);
    d_logn.ensure(h_logn.size());
    HIPCHK(hipMemcpyAsync(d_logn.p, h_logn.data(), h_logn.size() * 8, hipMemcpyHostToDevice, stream));
    d_c.ensure(n);
    HIPCHK(hipStreamSynchronize(stream));
    have_state = false;
    P = 0;
    return kOk;
  }

  int set_state(const int32_t* c_i, int K_, const double* cen, const double* sig) {
    if (!n) { err = "set_data first"; return kArg; }
    if (K_ < 0) { err = "K < 0"; return kArg; }
    K = K_;
    h_c.assign(c_i, c_i + n);
    h_center.assign((size_t)K * d, 0);
    h_sigma.assign(sig, sig + (size_t)K * d);
    for (size_t q = 0; q < (size_t)K * d; ++q) h_center[q] = (uint8_t)(int)cen[q];
    for (int i = 0; i < n; ++i)
      if (h_c[i] < 0) { err = "negative label"; return kArg; }
    recount();
    upload_labels();
    upload_clusters();
    have_state = true;
    return kOk;
  }

  int get_state(int32_t* c_i, int32_t* Kout, double* cen, double* sig, int cap) {
    if (!have_state) { err = "no state"; return kArg; }
    download_labels();
    if (c_i) std::memcpy(c_i, h_c.data(), (size_t)n * 4);
    if (Kout) *Kout = K;
    if (K > cap && (cen || sig)) { err = "cap too small"; return kArg; }
    for (size_t q = 0; q < (size_t)K * d; ++q) {
      if (cen) cen[q] = (double)h_center[q];
      if (sig) sig[q] = h_sigma[q];
    }
    return kOk;
  }

  // ------------------------------------------------------------------ pool
  void upload_pool() {
    std::vector<uint8_t> pc((size_t)P * dp, 0);
    std::vector<double> pt((size_t)P * 2 * d);
    std::vector<uint64_t> pb((size_t)P * bw);
    parallel_for(P, [&](int64_t a, int64_t b) {
      for (int64_t e = a; e < b; ++e) {
        tables_for(&h_pool_c[(size_t)e * d], &h_pool_s[(size_t)e * d], &pc[(size_t)e * dp], &pt[(size_t)e * 2 * d]);
        bounds_for(&h_pool_c[(size_t)e * d], &pt[(size_t)e * 2 * d], &pb[(size_t)e * bw]);
      }
    });

    d_pool_codes.ensure(pc.size());
    d_pool_tab.ensure(pt.size());
    d_pool_bnd.ensure(pb.size());
    HIPCHK(hipMemcpyAsync(d_pool_codes.p, pc.data(), pc.size(), hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(d_pool_tab.p, pt.data(), pt.size() * 8, hipMemcpyHostToDevice, stream));
    HIPCHK(hipMemcpyAsync(d_pool_bnd.p, pb.data(), pb.size() * 8, hipMemcpyHostToDevice, stream));
    build_pool_heads();
    HIPCHK(hipStreamSynchronize(stream));
  }

  int set_pool(const double* cen, const double* sig, int64_t P_) {
    if (!n) { err = "set_data first"; return kArg; }
    if (P_ <= 0 || P_ > 0x7fffffff) { err = "pool size must be in 1..2^31-1"; return kArg; }
    P = P_;
    pool_on_device = false;
    h_pool_c.resize((size_t)P * d);
    h_pool_s.assign(sig, sig + (size_t)P * d);
    for (size_t q = 0; q < (size_t)P * d; ++q) h_pool_c[q] = (uint8_t)(int)cen[q];
    upload_pool();
    return kOk;
  }

  // la:74-77 / la:124-128: per entry D centers then D sigmas, from the context stream.
  // The device generator (pool_gen.hpp) when the attributes qualify and the host libm is
  // the one glibc_math.hpp reproduces; the sequential host generator otherwise (or with
  // debug bit 6).  Both leave the same pool and the same stream position.
  int generate_pool(int64_t P_) {
    if (!n) { err = "set_data first"; return kArg; }
    if (P_ <= 0 || P_ > 0x7fffffff) { err = "pool size must be in 1..2^31-1"; return kArg; }
    auto t0 = std::chrono::steady_clock::now();
    int st = -1;
    if (!(debug & 64) && glibc_selfcheck()) st = generate_pool_device(P_);
    if (st < 0) st = generate_pool_host(P_);
    stats.pool_calls++;
    stats.pool_entries += P_;
    stats.t_pool_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return st;
  }

  int generate_pool_host(int64_t P_) {
    P = P_;
    pool_on_device = false;
    h_pool_c.resize((size_t)P * d);
    h_pool_s.resize((size_t)P * d);
    for (int64_t e = 0; e < P; ++e) {
      sample_center_uniform(&h_pool_c[(size_t)e * d]);
      int st = sample_sigma(v.data(), w.data(), &h_pool_s[(size_t)e * d]);
      if (st) { err = "rhig failed in pool generation"; return st; }
    }
    upload_pool();
    return kOk;
  }

  // The replicas of exp/log must equal this host's libm (they are the device's only way to
  // round like the reference); checked once per process.
  static bool glibc_selfcheck() {
    static const bool ok = [] {
      Rng r;
      r.set_seed(424242u);
      for (int k = 0; k < 200000; ++k) {
        const double u = r.unif();
        const double xs[4] = {u, u / (1.0 - u), 80.0 * u - 40.0, 0.9 + 0.2 * u};
        for (double x : xs) {
          const double a = std::exp(x), b = glibc::exp_h(x), c = std::log(x), e = glibc::log_h(x);
          if (std::memcmp(&a, &b, 8) != 0 || std::memcmp(&c, &e, 8) != 0) return false;
        }
      }
      return true;
    }();
    return ok;
  }

  // Returns -1 when the device generator does not apply (the caller falls back).
  int generate_pool_device(int64_t P_) {
    using clk = std::chrono::steady_clock;
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    if (!pg.planned) {
      pg.plan = pool_plan(d, att.data(), v.data(), w.data());
      pg.planned = true;
      if (pg.plan.ok) {
        const auto& pl = pg.plan;
        pg.cls.ensure(pl.cls.size());
        HIPCHK(hipMemcpy(pg.cls.p, pl.cls.data(), pl.cls.size() * sizeof(PoolClass), hipMemcpyHostToDevice));
        std::vector<int> runs(pl.run_cls);
        runs.insert(runs.end(), pl.run_len.begin(), pl.run_len.end());
        pg.runs.ensure(runs.size());
        HIPCHK(hipMemcpy(pg.runs.p, runs.data(), runs.size() * 4, hipMemcpyHostToDevice));
        pg.att.ensure(d);
        HIPCHK(hipMemcpy(pg.att.p, att.data(), (size_t)d * 4, hipMemcpyHostToDevice));
        pg.gtab.ensure(512);
        HIPCHK(hipMemcpy(pg.gtab.p, glibc::kGlibcExpTab, 256 * 8, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(pg.gtab.p + 256, glibc::kGlibcLogTab, 256 * 8, hipMemcpyHostToDevice));
        pg.err.ensure(1);
        pg.h_err.ensure(1);
      }
    }
    if (!pg.plan.ok) return -1;
    const PoolPlan& pl = pg.plan;
    const int nc = (int)pl.cls.size();

    rng_sync();
    if (rng.mti == 625) {   // never seeded: R's MT_sgenrand(4357) on the first draw
      uint32_t seed = 4357;
      for (int i = 0; i < 624; i++) {
        rng.mt[i] = seed & 0xffff0000u;
        seed = 69069u * seed + 1u;
        rng.mt[i] |= (seed & 0xffff0000u) >> 16;
        seed = 69069u * seed + 1u;
      }
      rng.mti = 624;
    }
    const int mti0 = rng.mti;
    const int64_t head = mti0 >= 624 ? 0 : 624 - mti0;
    pg.h_init.ensure(624);
    pg.init.ensure(624);
    std::memcpy(pg.h_init.p, rng.mt, sizeof(rng.mt));
    // the pool's old arrays may still be read by queued kernels: all work is on `stream`
    HIPCHK(hipMemcpyAsync(pg.init.p, pg.h_init.p, 624 * 4, hipMemcpyHostToDevice, stream));

    for (int attempt = 0; attempt < 3; ++attempt) {
      auto t0 = clk::now();
      const int64_t count = pool_slice_len(pl, P_, 1.0 + 0.25 * attempt) + 624;
      // slice generator: 256 workgroups with their own jump tables, or one for short slices
      const int G = 256;
      const bool multi = count >= (int64_t)G * 624 * 8;
      if (multi && (pg.G != G || count + head > (int64_t)624 * G * pg.bpg)) {
        const int bpg = (int)((count * 9 / 8 + 624 * G - 1) / (624 * G));
        if (!build_jump(pg.jpoly, pg.jidx, pg.joff, G, bpg)) return -1;
        pg.G = G;
        pg.bpg = bpg;
      }
      pg.raw.ensure(count);
      const int nblocks = count > head ? (int)((count - head + 623) / 624) : 0;
      MtGenArgs ma{pg.init.p, mti0, count, pg.raw.p, nullptr, nblocks, 0x7fffffff,
                   multi ? pg.jpoly.p : nullptr, pg.jidx.p, pg.joff.p, pg.bpg, multi ? G : 1};
      HIPCHK(launch_mt_gen(ma, stream));
      HIPCHK(hipStreamSynchronize(stream));
      auto tm = clk::now();

      const int64_t nwords = (count + 127) / 128;
      pg.bm.ensure((size_t)nc * 2 * nwords);
      // d even: every entry and every run starts at an even position, so only the even tables
      // are read (pool_gen.hpp)
      const int par_mask = (d % 2 == 0) ? 1 : 3;
      PoolAcceptArgs aa{pg.raw.p, count, nc, pg.cls.p, pg.bm.p, nwords, pg.gtab.p, par_mask};
      HIPCHK(launch_pool_accept(aa, stream));
      HIPCHK(hipStreamSynchronize(stream));
      auto t1 = clk::now();
      // entry starts by segments (k_pool_seg*, pool_gen.hpp PoolSegPlan); the serial host
      // parse when the chain leaves a window (an entry longer than mean + 14 sd)
      const PoolSegPlan sp = pool_seg_plan(pl, d, count);
      const size_t cells = (size_t)sp.nchunks * sp.ncand;
      pg.T.ensure(cells);
      pg.gj.ensure((size_t)sp.ngroups * sp.ncand);
      pg.gn.ensure((size_t)sp.ngroups * sp.ncand);
      pg.cidx.ensure(sp.nchunks);
      pg.cE.ensure(sp.nchunks);
      pg.aux.ensure(1);
      pg.starts.ensure(P_ + 1);
      pg.h_starts.ensure(P_ + 1);
      HIPCHK(hipMemsetAsync(pg.err.p, 0, 4, stream));
      HIPCHK(hipMemsetAsync(pg.cidx.p, 0xFF, (size_t)sp.nchunks * 4, stream));
      const int nr = (int)pl.run_cls.size();
      PoolSegArgs sa{pg.bm.p, nwords, d, PoolRuns{nr, pg.runs.p, pg.runs.p + nr}, sp, P_, pg.T.p, pg.gj.p, pg.gn.p,
                     pg.cidx.p, pg.cE.p, pg.aux.p, pg.starts.p, pg.err.p};
      HIPCHK(launch_pool_seg(sa, stream));
      HIPCHK(hipMemcpyAsync(pg.h_err.p, pg.err.p, 4, hipMemcpyDeviceToHost, stream));
      HIPCHK(hipMemcpyAsync(&pg.h_starts.p[P_], pg.starts.p + P_, 8, hipMemcpyDeviceToHost, stream));
      HIPCHK(hipStreamSynchronize(stream));
      int64_t end = pg.h_starts.p[P_];
      const int werr = *pg.h_err.p;
      if (werr & 8) end = -1;
      if (!(werr & 8) && (werr & 4 || (debug & 268435456))) {
        // the chain left a window (or debug bit 28): the sequential walk
        pg.walk_fallbacks++;
        stats.pool_walk_fallbacks++;
        pg.h_bm.ensure((size_t)nc * 2 * nwords);
        HIPCHK(hipMemcpyAsync(pg.h_bm.p, pg.bm.p, (size_t)nc * 2 * nwords * 8, hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        PoolRuns R{(int)pl.run_cls.size(), pl.run_cls.data(), pl.run_len.data()};
        end = pool_parse(pg.h_bm.p, nwords, d, R, 0, 0, P_, pg.h_starts.p);
        if (end >= 0) {
          pg.h_starts.p[P_] = end;
          HIPCHK(hipMemcpyAsync(pg.starts.p, pg.h_starts.p, (size_t)(P_ + 1) * 8, hipMemcpyHostToDevice, stream));
        }
      }
      auto t2 = clk::now();
      stats.t_pool_mt_ms += ms(t0, tm);
      stats.t_pool_accept_ms += ms(tm, t1);
      stats.t_pool_parse_ms += ms(t1, t2);
      if (end < 0 || end + 624 > count) continue;      // slice too short: a longer one

      P = P_;
      d_pool_codes.ensure((size_t)P * dp);
      d_pool_tab.ensure((size_t)P * 2 * d);
      d_pool_bnd.ensure((size_t)P * bw);
      d_pool_sig.ensure((size_t)P * d);
      HIPCHK(hipMemsetAsync(pg.err.p, 0, 4, stream));
      PoolValueArgs va{pg.raw.p, count, pg.starts.p, P, d, dp, wb, Ws, bw, pg.att.p, (int)pl.run_cls.size(),
                       pg.runs.p, pg.runs.p + pl.run_cls.size(), pg.cls.p, pg.bm.p, nwords, pg.gtab.p,
                       d_pool_codes.p, d_pool_tab.p, d_pool_sig.p, d_pool_bnd.p, pg.err.p};
      HIPCHK(launch_pool_values(va, stream));
      build_pool_heads();
      HIPCHK(hipMemcpyAsync(pg.h_err.p, pg.err.p, 4, hipMemcpyDeviceToHost, stream));

      // the stream continues after `end` draws: mti and the block array (untempered outputs)
      int64_t blk;
      int mti;
      if (end < head) {
        blk = 0;
        mti = mti0 + (int)end;
      } else {
        const int64_t b = 1 + (end - head) / 624, k = (end - head) % 624;
        blk = k == 0 ? b - 1 : b;
        mti = k == 0 ? 624 : (int)k;
      }
      pg.h_tail.ensure(624);
      if (blk > 0)
        HIPCHK(hipMemcpyAsync(pg.h_tail.p, pg.raw.p + head + (blk - 1) * 624, 624 * 4, hipMemcpyDeviceToHost,
                              stream));
      HIPCHK(hipStreamSynchronize(stream));
      stats.t_pool_values_ms += ms(t2, clk::now());
      if (*pg.h_err.p) {
        err = "device pool generator: inconsistent walk";
        return kDevice;
      }
      if (blk > 0)
        for (int t = 0; t < 624; ++t) rng.mt[t] = mt_untemper(pg.h_tail.p[t]);
      rng.mti = mti;
      rng.pos += (uint64_t)end;
      pool_on_device = true;
      h_pool_c.clear();
      h_pool_c.shrink_to_fit();
      h_pool_s.clear();
      h_pool_s.shrink_to_fit();
      stats.pool_device_calls++;
      return kOk;
    }
    return -1;
  }

  void get_pool(double* centers, double* sigma) {
    const size_t nn = (size_t)P * d;
    if (!pool_on_device) {
      for (size_t q = 0; q < nn; ++q) {
        if (centers) centers[q] = h_pool_c[q];
        if (sigma) sigma[q] = h_pool_s[q];
      }
      return;
    }
    if (centers) {
      std::vector<uint8_t> c((size_t)P * dp);
      HIPCHK(hipMemcpyAsync(c.data(), d_pool_codes.p, c.size(), hipMemcpyDeviceToHost, stream));
      HIPCHK(hipStreamSynchronize(stream));
      for (int64_t e = 0; e < P; ++e)
        for (int j = 0; j < d; ++j) centers[(size_t)e * d + j] = c[(size_t)e * dp + j];
    }
    if (sigma) {
      HIPCHK(hipMemcpyAsync(sigma, d_pool_sig.p, nn * 8, hipMemcpyDeviceToHost, stream));
      HIPCHK(hipStreamSynchronize(stream));
    }
  }

  // Centers and sigmas of pool entry e (device pools are read back on demand).
  void pool_entry(int64_t e, uint8_t* cen, double* sig) {
    if (!pool_on_device) {
      std::memcpy(cen, &h_pool_c[(size_t)e * d], d);
      std::memcpy(sig, &h_pool_s[(size_t)e * d], (size_t)d * 8);
      return;
    }
    HIPCHK(hipMemcpyAsync(cen, d_pool_codes.p + (size_t)e * dp, d, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipMemcpyAsync(sig, d_pool_sig.p + (size_t)e * d, (size_t)d * 8, hipMemcpyDeviceToHost, stream));
  }

  // ------------------------------------------------------------------ Neal-8 sweep
  bool mcount_clear = false;
  bool summary_by_scatter = false;     // the pipelined scatter wrote this round's summaries (pre_enqueue)
  // Buffers of a sweep (sized for n).
  void sweep_buffers(bool track, int m) {
    const int nb_max = (n + kBlock - 1) / kBlock;
    d_margin.ensure(n);
    d_rowpos.ensure(n);
    d_list.ensure((size_t)nb_max * kBlock);
    d_cnt.ensure((size_t)nb_max * (kBlock / 16));   // list blocks of 16 points (k_prepass_wide chunks)
    d_boff.ensure((size_t)nb_max * (kBlock / 16));
    d_dense.ensure((size_t)nb_max * kBlock);
    d_dense_total.ensure(1);
    d_spec.ensure((size_t)nb_max * kBlock);
    d_spec_rad.ensure((size_t)nb_max * kBlock);
    d_rq.ensure((size_t)nb_max * kBlock);
    // the device-wide resolver's scratch for a grid of every CU (allocated here, not at its
    // first launch: a hipMalloc inside a timed sweep cost ~8 ms)
    {
      const int cus = device_cus();
      d_fpg.ensure(fpg_words(2 * cus));
      // and the occupancy of the kernels of the unconverged regime, at every resolver slot
      // capacity this chain can take next
      for (int lc = 2; lc <= std::min(scap, 64); ++lc)
        if (fpg_grid(lc, m) == 0) {
          const int mg = warm_sweep_kernels(lc, m);
          fpg_grid(lc, m) = mg >= 2 ? mg : -1;
        }

    }
    if (track) {
      d_mlog.ensure((size_t)3 * n);
      d_mcount.ensure(1);
      mcount_clear = true;            // by the next launch's k_cluster_summary
    }
  }

  // One launch of the sweep from point p with nslots slots: cluster summary, prepass, exact
  // rows, resolver, control copy, and the sweep-end kernels behind it (they act only if
  // this launch completes the sweep).  kOk or kArg (resolver state too large for LDS).
  // part: kRoundAll, kRoundPrefix (up to the exact rows: kernels that write scratch only, so
  // a prepared sweep can start on the device and still be dropped), kRoundResolve (the rest,
  // after a prefix launched with the same arguments and no state change in between).
  enum { kRoundAll = 0, kRoundPrefix = 1, kRoundResolve = 2 };
  static constexpr int kFpMinListed = 64;
  static constexpr int kFpgMinListed = 1024;   // listed points of the previous launch for k_resolve_fpg (two chunks)
  static constexpr int kMassNoSpec = 65536;    // expected listed points above which no snapshot draws are made
  // HDPM_FPG_MIN: the listed points (expected) from which launches take k_resolve_fpg (A/B)
  static int fpg_min_listed() {
    static const int v = [] {
      const char* e = std::getenv("HDPM_FPG_MIN");
      return e ? std::max(1, std::atoi(e)) : (int)kFpgMinListed;
    }();
    return v;
  }
  static constexpr int kDenseMinPoints = 4096;  // dense listing only for launches over at least this many points
  // the state fits the dense path: the fixed-point resolvers and a mass exact-rows kernel
  // (kernels.hip launch_exact_rows: the thread-per-point kernel's LDS tables, or the
  // wave-per-point kernel's)
  bool dense_list_fits(int m, int nslots) const {
    const int lcap = std::min(scap, nslots + 2);
    if (!fp_eligible(K + m, lcap) || (debug & (2048 | 8))) return false;
    const size_t lanes_lds = (size_t)K * (2 * (size_t)d * 8 + (size_t)nq * 16);
    const size_t mass_lds = (size_t)K * 2 * d * 8 + (size_t)8 * m * d * 8 + (size_t)K * nq * 16 + (size_t)8 * nq * 16;
    return (nq <= 8 && K <= 64 && lanes_lds <= 64 * 1024) || mass_lds <= 96 * 1024;
  }
  static bool fp_unsettled_unif() {
    static const bool on = [] {
      const char* e = std::getenv("HDPM_FP_UNSETTLED_UNIF");
      return !(e && std::atoi(e) == 0);
    }();
    return on;
  }
  // HDPM_DENSE_DIRECT=0: dense launches still run the prepass (A/B)
  static bool dense_direct_on() {
    static const bool on = [] {
      const char* e = std::getenv("HDPM_DENSE_DIRECT");
      return !(e && std::atoi(e) == 0);
    }();
    return on;
  }
  // HDPM_LAT_BOUND=0: every latent column exact in the level-table rows (A/B)
  static bool lat_bound_on() {
    static const bool on = [] {
      const char* e = std::getenv("HDPM_LAT_BOUND");
      return !(e && std::atoi(e) == 0);
    }();
    return on;
  }
  static bool lv_spec_on() {
    static const bool on = [] {
      const char* e = std::getenv("HDPM_LV_SPEC");
      return !(e && std::atoi(e) == 0);
    }();
    return on;
  }
  // HDPM_DENSE_LIST=0: no dense listing (A/B)
  static bool dense_list_on() {
    static const bool on = [] {
      const char* e = std::getenv("HDPM_DENSE_LIST");
      return !(e && std::atoi(e) == 0);
    }();
    return on;
  }
  bool fp_eligible(int E, int lcap) const {
    return E <= 64 && lcap <= 64 && !(debug & (1 | 4096 | 8192 | 8388608));
  }
  // pg: a sweep enqueued ahead (pre_enqueue) -- its kernels take the gate and the draws
  // from pg, its control block is cpar; no timing events, no counters.
  int launch_round(int p, int nslots, int m, const uint32_t* d_sweep_raw, bool track, int part = kRoundAll,
                   PipeGate* pg = nullptr, int cpar = -1) {
    const double dmax = 0.25;
    if (cpar < 0) cpar = par;
    ensure_slots(nslots + 2);
    // points this launch will likely list: the previous launch's density over [p, n) (a
    // restart late in a sweep lists few points; the next sweep's first launch lists many)
    // A context's first launch has no previous density: it is taken as dense (every point listed)
    // where the mass exact-rows kernels and the fixed-point resolvers fit -- from a random start
    // (the scripts' L = 20) nearly every point is uncertain, and a first sweep sized for a
    // converged chain ran on one workgroup (~220 ms at C5); a converged chain pays one dense
    // sweep once.
    const bool dense_fits = dense_list_fits(m, nslots);
    const int el = last_density < 0 ? (dense_fits ? n - p : -1)
                                    : (int)std::min<double>((double)n, last_density * (double)(n - p) + 0.5);
    // Dense launches (more than half the points expected uncertain) list every point: the
    // resolver then decides all of them and never re-tests an unlisted one against the count
    // drift -- a re-test failure restarted the launch, and its prepass and exact rows, at that
    // point (C5 from a random start: ~118 certified points per sweep restarted ~700k rows)
    const bool dense_list = dense_fits && el >= kDenseMinPoints && 2 * (int64_t)el >= (int64_t)(n - p) &&
                            !(debug & 1) && dense_list_on();
    // the resolver writes its control block and summary straight into host memory
    if (h_ctl.n < 2 * ctl_stride()) h_ctl.ensure(2 * ctl_stride(), hipHostMallocCoherent);
    for (auto& e : ev_res)
      if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // HIP events between kernels cost a dispatch gap each: the prepass is timed on every
    // 8th launch (all launches, and the other kernels too, in the diagnostic modes)
    if (part != kRoundResolve && !pg) {
      round_fine = (debug & (2 | 32 | 512)) != 0;
      round_timed = round_fine || (launch_count++ % 8 == 0);
    }
    const int S = nslots;
    if (S + m > Ecap) {
      Ecap = std::max(S + m, std::max(2 * Ecap, 32));
      d_L.ensure((size_t)Ecap * n);
    }
    const int E = K + m;
    const double T = 54.0 * M_LN2 + std::log((double)E) + 0.5;
    PrepassArgs pa;
    pa.gate = pg ? &pg->gate : nullptr;
    pa.raw_ptr = pg ? &pg->raw : nullptr;
    // with the device update_phi beside the sweep (dspec), three of the four prepass
    // workgroups per CU: the update's group kernel starts beside the prepass instead of behind
    // it (C4: 6,170 -> 6,538 it/s; the iteration is the update's chain there)
    pa.wide_per_cu = dspec_on() ? 3 : 0;
    pa.codes_t = d_codes_t.p; pa.n = n; pa.d = d; pa.nq = nq; pa.mmax = mmax;
    pa.c = d_c.p; pa.counts = d_counts.p; pa.slot_of_label = d_sol.p; pa.K = K; pa.S = S;
    pa.slots = ParamTables{d_slot_codes.p, d_slot_tab.p};
    pa.pool = ParamTables{d_pool_codes.p, d_pool_tab.p};
    pa.P = P; pa.raw = d_sweep_raw; pa.m = m; pa.logn = d_logn.p; pa.logfac = std::log(gamma / m);
    pa.xbs = d_xbs.p; pa.Ws = Ws; pa.wb = wb; pa.slot_bnd = d_slot_bnd.p; pa.pool_bnd = d_pool_bnd.p; pa.bw = bw;
    pa.pool_head = (head_fits(wb, Ws) && !(debug & 1024)) ? d_pool_head.p : nullptr;
    pa.head_ha = head_ha;
    pa.head_hb = head_hb;
    d_csum.ensure((size_t)std::max(K, 1) * (bw + 2));
    pa.csum = d_csum.p;

    pa.thresh = ((debug & 1) || dense_list) ? INFINITY : T + 2.0 * dmax;
    pa.thresh_ref = T + 2.0 * dmax;
    // certification by the draw's uniform only while the chain is settled: after a launch
    // that exceeded its drift budget, restarted or decided many points itself, uniform-
    // certified points (no exact rows) would fail re-verification and restart the launch
    // (the fixed-point resolver re-tests and restarts cheaply enough to keep the uniform
    // certification after many exact decisions; debug bit 24 lists every point there too)
    const bool fp_next = fp_eligible(K + m, std::min(scap, nslots + 2)) &&
                         (el < 0 || el >= kFpMinListed || (debug & 33554432));
    const bool many_exact = last_exact >= kResolveBlkMin && (!fp_next || (debug & 16777216));
    // The fixed-point resolvers keep the uniform's certification after an unsettled launch
    // (a restart behind a new cluster, a drift past the budget): a point it certified that no
    // longer holds is re-tested and restarts the launch, which these resolvers do cheaply,
    // while listing every uncertain point by margin alone cost C2's restart launches ~5x the
    // points (3,106 vs ~530) and ~300 us each (HDPM_FP_UNSETTLED_UNIF=0: margins only, as the
    // one-wave resolvers need)
    const bool unsettled_margins = last_unsettled && !(fp_next && fp_unsettled_unif());
    pa.dmax2_ref = ((debug & (1 | 262144)) || unsettled_margins || many_exact) ? INFINITY : 2.0 * dmax;
    pa.dmax2 = dense_list ? INFINITY : pa.dmax2_ref;
    if (dense_list && !pg && part != kRoundResolve) stats.dense_launches++;
    pa.L = d_L.p; pa.rowpos = d_rowpos.p; pa.margin = d_margin.p; pa.list = d_list.p; pa.cnt = d_cnt.p;
    pa.dense = d_dense.p; pa.dense_total = d_dense_total.p; pa.boff = d_boff.p;
    // snapshot draws (k_exact_rows*: the resolver's first-round guesses and kept draws) except
    // when nearly every point is listed: the device-wide resolver then draws all of them in
    // its first round anyway, and the mass exact-rows kernel is ~20% faster without them
    // (with the level-table exact rows the snapshot draws are made behind the rows by
    // k_snap_draws, a thread per point, also for dense launches; HDPM_LV_SPEC=0: not there)
    pa.spec_lv = lv_spec_on() ? 1 : 0;
    // latents far below the clusters kept as head bounds by the level-table exact rows; only
    // for the fixed-point resolvers (their draws and the serial path take the bounds,
    // kernels.hip latent_fix), with pool-entry heads
    pa.lbound = (fp_next && pa.pool_head && m <= 32 && lat_bound_on()) ? 1 : 0;
    d_lmask.ensure((size_t)((n + kBlock - 1) / kBlock) * kBlock);
    pa.lmask = d_lmask.p;
    pa.lat_negl = lat_negl;
    pa.exact_pref = exact_pref;
    // a dense launch needs no bounds: its list is every point (k_dense_list)
    pa.dense_direct = dense_list && dense_direct_on() ? 1 : 0;
    pa.spec = ((debug & 8) || (el >= kMassNoSpec && !pa.spec_lv)) ? nullptr : d_spec.p;
    pa.spec_rad = d_spec_rad.p;
    pa.rq = d_rq.p;
    pa.p0 = p;
    pa.exact_wave = (debug & 2048) ? 1 : 0;
    pa.exact_grid = el < 0 ? 0 : std::min(1536, std::max(64, el + 64));
    pa.exact_scan = el >= 4096 ? 1 : 0;
    pa.wide = (debug & 16384) ? 0 : 1;
    pa.zero = nullptr;
    d_wide_ctr.ensure(4);
    pa.wide_ctr = d_wide_ctr.p;      // cleared by k_cluster_summary (below: K > 0)
    if (K == 0 && part != kRoundResolve) HIPCHK(hipMemsetAsync(d_wide_ctr.p, 0, 16, stream));
    if (mcount_clear && part != kRoundResolve) {
      if (K > 0) pa.zero = d_mcount.p;
      else HIPCHK(hipMemsetAsync(d_mcount.p, 0, 4, stream));
      mcount_clear = false;
    }
    const int nblocks = (n - p + kBlock - 1) / kBlock;
    const bool timed = round_timed && !pg, fine = round_fine && !pg;
    if (pg) {
      pre_timed[cpar] = launch_count++ % 8 == 0;
      for (auto& e : ev_pp[cpar])
        if (!e) HIPCHK(hipEventCreate(&e));
    }
    if (part != kRoundResolve) {
      if (!summary_by_scatter) HIPCHK(launch_cluster_summary(pa, stream));
      if (timed) HIPCHK(hipEventRecord(ev[0], stream));
      if (pg && pre_timed[cpar]) HIPCHK(hipEventRecord(ev_pp[cpar][0], stream));
      if (pa.dense_direct) HIPCHK(launch_dense_list(pa, stream));
      else HIPCHK(launch_prepass(pa, nblocks, stream));
      mark("r.prepass");
      if (!pg) {
        stats.prepass_points += n - p;
        round_points = n - p;
      }
      if (timed) HIPCHK(hipEventRecord(ev[1], stream));
      if (pg && pre_timed[cpar]) HIPCHK(hipEventRecord(ev_pp[cpar][1], stream));
      int xpath = 0;
      HIPCHK(launch_exact_rows(pa, nblocks, stream, &xpath));
      last_xpath = xpath;
      if (!pg) {
        if (xpath == 1) stats.exact_mass_launches++;
        if (xpath == 2 || xpath == 3) stats.exact_lanes_launches++;
      }
      mark("r.exact");
      if (fine) HIPCHK(hipEventRecord(ev[5], stream));
    }

    ResolveArgs ra;
    ra.gate = pa.gate;
    ra.raw_ptr = pa.raw_ptr;
    ra.dry = 0;
    ra.n = n; ra.d = d; ra.dp = dp; ra.m = m; ra.P = P;
    ra.c = d_c.p; ra.counts = d_counts.p; ra.slot_of_label = d_sol.p; ra.label_of_slot = d_los.p;
    ra.slot_src = d_src.p; ra.slot_codes = d_slot_codes.p; ra.slot_tab = d_slot_tab.p;
    ra.pool = pa.pool; ra.raw = d_sweep_raw; ra.logn = d_logn.p; ra.logfac = pa.logfac;
    ra.L = d_L.p; ra.rowpos = d_rowpos.p; ra.slot_bnd = d_slot_bnd.p; ra.pool_bnd = d_pool_bnd.p; ra.bw = bw;
    ra.S = S; ra.margin = d_margin.p; ra.list = d_list.p; ra.dense = d_dense.p; ra.dense_total = d_dense_total.p;
    ra.spec = pa.spec;
    ra.spec_rad = pa.spec_rad;
    ra.rq = pa.rq;
    ra.nblocks = nblocks; ra.p0 = p; ra.T = T; ra.dmax = dmax; ra.scap = scap; ra.K = K;
    ra.lcap = std::min(scap, nslots + 2);
    ra.nslots = nslots; ra.ctl = ctl_at(cpar); ra.summary = (int*)ctl_at(cpar) + kCtlInts; ra.force_exact = (debug & 1);
    ra.prof = nullptr;
    ra.mlog = track ? d_mlog.p : nullptr;
    ra.mcount = track ? d_mcount.p : nullptr;
    ra.freq = track ? d_freq.p : nullptr;
    ra.fstride = d * mmax;
    if ((debug & 2) && !pg) {
      d_rprof.ensure(16);
      ra.prof = d_rprof.p;
    }
    // block mode when in the previous launch many uncertain points had to be decided one by
    // one (their snapshot draws no longer held: an unconverged chain, or clusters appearing
    // and vanishing); LIST mode passes over the rest in one ballot per 64
    ra.blocks = (K + m <= 64 && nslots <= 64 && !(debug & 4096) && !(debug & 1) &&
                 ((debug & 8192) || last_exact >= kResolveBlkMin)) ? 1 : 0;
    // the fixed-point resolver whenever the state fits it (debug bit 23: the one-wave LIST /
    // block modes; bits 12 / 13 select those modes and keep them)
    // (a launch whose predecessor listed only a few points -- a converged chain -- keeps the
    // one-wave LIST resolver: its fixed cost is half the fixed-point kernel's, ~7 vs ~13 us at C5)
    ra.fp = (fp_eligible(K + m, ra.lcap) && (el < 0 || el >= kFpMinListed || (debug & 33554432)))
                ? 1 : 0;
    if (ra.fp) ra.blocks = 0;
    ra.debug_fp = (debug & 67108864) ? 1 : 0;
    // the device-wide fixed-point resolver (k_resolve_fpg) after a launch that listed many
    // points: one 512-point chunk per workgroup, a workgroup per CU (debug bit 29: one workgroup)
    ra.fpg = 0;
    ra.fpg_buf = nullptr;
    // (k_snap_draws, behind the level-table exact rows, counted them)
    ra.uncertain = (pa.dense_direct && pa.spec && last_xpath == 3) ? d_wide_ctr.p + 2 : nullptr;
    ra.lmask = (pa.lbound && last_xpath == 3) ? d_lmask.p : nullptr;
    ra.codes_t = d_codes_t.p;
    ra.lat_negl = lat_negl;
    ra.all_listed = pa.dense_direct;
    ra.nq = nq;
    ra.fpg_limit = fpg_limit_ticks;
    ra.fpg_fail = fpg_fail_at;
    const bool fpg_skipped = fpg_skip && part != kRoundPrefix;
    if (fpg_skipped) fpg_skip = false;
    if (ra.fp && !fpg_skipped && (el >= fpg_min_listed() || (debug & 1073741824)) && !(debug & 536870912) &&
        ra.lcap <= 64) {
      int& mg = fpg_grid(ra.lcap, m);
      if (mg == 0) {
        mg = resolve_fpg_max_grid(ra.lcap, m);
        if (mg < 2) mg = -1;
      }
      if (mg > 0 && resolve_fpg_smem_bytes(ra.lcap, m) <= 160 * 1024) {
        const int G = std::min(mg, std::max(2, (std::max(el, 0) + 511) / 512));
        d_fpg.ensure(fpg_words(G));
        HIPCHK(hipMemsetAsync(d_fpg.p, 0, (size_t)kFpgZeroWords * 4, stream));
        ra.fpg = G;
        ra.fpg_buf = d_fpg.p;
        if (!pg) stats.fpg_launches++;
      }
    }
    if (part != kRoundPrefix && !pg) {
      last_fp = ra.fp != 0;
      last_fpg = ra.fpg;
    }
    if (resolve_smem_bytes(ra.lcap, m, ra.blocks) > 160 * 1024) {
      err = "too many clusters for the resolver (K > ~2300)";
      return kArg;
    }
    if (part == kRoundPrefix) return kOk;
    mark("r.args");
    if (!kernels_warm && !pg) {
      // the kernels this chain may reach only later, each launched once behind a closed gate
      d_warm.ensure(32);
      HIPCHK(hipMemsetAsync(d_warm.p, 0, 32 * sizeof(int), stream));
      HIPCHK(warm_launch_kernels(pa, ra, d_warm.p, d_warm.p + 16, stream));
      kernels_warm = true;
    }
    HIPCHK(launch_resolve(ra, stream));
    mark("r.resolve");
    if (fine) HIPCHK(hipEventRecord(ev[2], stream));
    HIPCHK(hipEventRecord(ev_res[cpar], stream));
    return kOk;
  }

  // The sweep end after a completed sweep with moves (a sweep without moves leaves labels,
  // counts, slot maps and frequency tables as they were): slot ids -> labels, the moves
  // applied to the frequency tables and these re-indexed to labels (copied out behind),
  // identity slot maps.  The kernels read the final launch's control block in host memory.
  void launch_sweep_end(int nslots, bool track) {
    const ResolveCtl* hctl = ctl_at(par);
    HIPCHK(launch_relabel(d_c.p, d_los.p, n, hctl, stream));
    if (track) {
      HIPCHK(launch_apply_moves(d_mlog.p, d_mcount.p, (int)std::min<int64_t>(n, 4096), d_codes_t.p, d, nq, mmax,
                                d_freq.p, hctl, n, scap, stream));
      HIPCHK(launch_freq_gather(d_freq.p, d_sol.p, std::min(scap, nslots + 2), d * mmax, d_freq2.p, hctl, n, stream));
      const size_t fwords = (size_t)std::min(scap, nslots + 2) * d * mmax;
      h_freq_next.ensure((size_t)scap * d * mmax);   // every slot count at once: no reallocation later
      HIPCHK(hipMemcpyAsync(h_freq_next.p, d_freq2.p, fwords * 4, hipMemcpyDeviceToHost, stream));
    }
    HIPCHK(launch_finish_sweep(d_counts.p, d_sol.p, d_los.p, d_src.p, scap, hctl, n, stream));
    // (the labels' copies on cstream wait for this: the resolver's end tells the host the sweep
    // is done, not that k_relabel has turned its slot ids into labels)
    if (!ev_labels) HIPCHK(hipEventCreateWithFlags(&ev_labels, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ev_labels, stream));
  }
  hipEvent_t ev_labels = nullptr;      // the last sweep end (launch_sweep_end) on `stream`

  // The next sweep prepared at the end of an iteration (prepare_next_sweep): its draws
  // reserved (their stream slice and update_phi's are copied out) and update_phi speculated
  // on the pool, while the caller returns and comes back to launch the sweep.  Any other
  // entry point cancels it (cancel_ahead): the job is joined and the stream rewound to
  // where the sweep would have started.
  struct Ahead {
    bool active = false;
    int m = 0;
    uint64_t lv = 0;
    Rng saved;
    const uint32_t* raw = nullptr;
    bool launched = false;             // round 0 of the sweep is already on the device
    bool prefix = false;               // round 0's prepass part is on the device (droppable)
    bool track = false;
    int par = 0;                       // control block of the prepared sweep
    bool piped = false;                // enqueued ahead (pre_enqueue / pipe_go)
  } ahead;

  // With `launch` (only when the caller runs the sweep next, no other call in between:
  // a launched sweep cannot be cancelled), round 0 of the sweep is launched too, so the
  // device goes on from this iteration's uploads without waiting for the host.
  void prepare_next_sweep(int m, bool launch) {
    if (ahead.active || !have_state || P <= 0 || m <= 0 || tables_dirty || (debug & (256 | 128 | 16))) return;
    if (!(freq_dev_valid && freq_version == labels_version)) return;
    rng_sync();
    mark("ahead.sync");
    ahead.saved = rng;
    ahead.raw = device_draws((int64_t)n * (m + 1));
    mark("ahead.draws");
    ahead.m = m;
    ahead.lv = labels_version;
    ahead.launched = false;
    ahead.prefix = false;
    ahead.piped = false;
    ahead.active = true;
    // the speculative update_phi first: its serial draws, not the device sweep, are the
    // longer path (timeline: launching the sweep first cost ~8% of the iteration rate);
    // debug bit 15 launches the sweep first
    const bool sweep_first = (debug & 32768) != 0;
    if (!sweep_first && host_spec()) {
      spec_launch();
      mark("ahead.spec");
    }
    flush_commit();                       // this iteration's tables, before the sweep that reads them
    if (!host_spec()) {
      dspec_launch();                     // after the scatter of this iteration's tables (ev_phd_free)
      mark("ahead.dspec");
    }
    if (resolve_smem_bytes(std::min(scap, K + 2), m, K + m <= 64 ? 1 : 0) <= 160 * 1024) {
      par ^= 1;                           // the prepared sweep's control block
      ahead.par = par;
      ahead.track = freq_dev_valid;
      sweep_buffers(ahead.track, m);
      mark("ahead.buf");
      // the whole round 0 when the caller runs the sweep next; otherwise its prepass part
      // only (scratch outputs: any other call can still drop the prepared sweep)
      if (launch) {
        if (launch_round(0, K, m, ahead.raw, ahead.track) == kOk) ahead.launched = true;
      } else if (!(debug & 131072)) {
        // hdpm_synchronize waits for the chain's work up to here, not for the prepared prefix
        HIPCHK(hipEventRecord(ev[7], stream));
        if (launch_round(0, K, m, ahead.raw, ahead.track, kRoundPrefix) == kOk) ahead.prefix = true;
      }
    }
    if (sweep_first && host_spec()) {
      spec_launch();
      mark("ahead.spec");
    }
  }
  void cancel_ahead() {
    pre_release();
    if (!ahead.active) return;
    ahead.active = false;
    if (ahead.launched) {
      // a launched sweep cannot be taken back: the chain state is no longer defined
      (void)hipStreamSynchronize(stream);
      have_state = false;
      err = "a prepared sweep was abandoned";
    }
    if (spec.ran) {
      if (!spec.joined && pj_open) (void)pj_finish();
      spec.ran = false;
    }
    dspec.ran = false;                   // (its device work completes unused)
    dnext.ran = false;
    phi_stream.n = 0;
    pend.active = false;
    rng = ahead.saved;
  }

  int last_sweep_rounds = 0, last_sweep_moves = -1;   // of the last sweep (pipe_go)

  // The next sweep, enqueued while the speculative update_phi of this one runs (its tables
  // are that update's, from the held staging buffer): a wait kernel, the tables' copy and
  // scatter, round 0 -- all gated on the device by k_pipe_wait.  The host decides after this
  // iteration's update_phi: pipe_go (the sweep completed in its one launch without a move
  // and the update came whole from the speculation) or pre_release.
  void pre_enqueue(int m, bool track) {
    const int q = 1 - par;
    // every buffer sized before the wait kernel is queued (a reallocation would synchronise)
    if (h_pipe.n < 2) h_pipe.ensure(2, hipHostMallocCoherent);
    d_pipe.ensure(2);
    sweep_buffers(track, m);
    __atomic_store_n(&h_pipe.p[q].flag, 0, __ATOMIC_RELEASE);
    __atomic_store_n(&h_pipe.p[q].dev, 0, __ATOMIC_RELEASE);
    h_pipe.p[q].raw = nullptr;
    h_pipe.p[q].raw_dev = nullptr;
    // the next sweep's draws start after this update's (about a slice): the windows that
    // overlap that stretch (not a window generation started for later sweeps)
    const bool dev = !host_spec();
    const uint64_t lo = dev ? dspec.pos : spec.pos;
    const uint64_t hi = lo + (uint64_t)(dev ? dspec.pl.need : 2 * phi_prefetch) + (uint64_t)n * (m + 1);
    int whole = -1;                      // the earliest window holding all of it
    for (int k = 0; k < 2; ++k) {
      const RngWindow& w = win[k];
      if (w.valid && w.epoch == rng.epoch && w.start_pos <= lo && hi <= w.start_pos + (uint64_t)w.count &&
          (whole < 0 || w.start_pos < win[whole].start_pos))
        whole = k;
    }
    for (int k = 0; k < 2; ++k) {
      pre.gen[k] = ~0ull;
      const RngWindow& w = win[k];
      if (whole >= 0 ? k == whole
                     : (w.valid && w.epoch == rng.epoch && w.start_pos < hi && lo < w.start_pos + (uint64_t)w.count)) {
        HIPCHK(hipStreamWaitEvent(stream, w.done, 0));
        pre.gen[k] = w.gen;
      }
    }
    // the device's own go (PipeAuto) when the speculated update is the fast path's: the wait
    // kernel goes behind the update's completion and reads its chain word
    static const bool auto_env_off = [] {
      const char* e = std::getenv("HDPM_PIPE_AUTO");
      return e && e[0] == '0';
    }();
    PipeAuto au{};
    if (dev && pipe_auto && !auto_env_off && dspec.ran && dspec.fast && dspec.chain && whole >= 0) {
      const RngWindow& w = win[whole];
      au = PipeAuto{dspec.chain, w.raw.p, (int64_t)w.start_pos, w.count, (int64_t)n * (m + 1), 1};
    }
    if (dev) HIPCHK(hipStreamWaitEvent(stream, dspec.ev, 0));   // (the update's tables, below)
    HIPCHK(launch_pipe_wait(&h_pipe.p[q], ctl_at(par), ctl_at(q), n, &d_pipe.p[q], pipe_limit_ticks, stream, au));
    pre.au = au.on != 0;
    pre.t_enq = std::chrono::steady_clock::now();   // the kernel's clock starts no earlier
    pre.active = true;
    pre.par = q;
    pre.dev = dev;
    pre.buf = dev ? -1 : spec.stage_buf;
    pre.m = m;
    pre.track = track;
    pre.round_ok = false;
    // the scatter also writes the round's cluster summaries (k_cluster_summary's work) from the
    // staged records: one launch fewer between the wait kernel and the prepass
    d_csum.ensure((size_t)K * (bw + 2));
    d_wide_ctr.ensure(4);
    int* zero = nullptr;
    if (mcount_clear && K > 0) {
      zero = d_mcount.p;
      mcount_clear = false;
    }
    if (dev) {
      // the speculative device update's tables (its staging buffer; the stream waited for it)
      HIPCHK(launch_scatter_clusters(dspec.stage, K, dp, d, bw, 1, d_slot_codes.p, d_slot_tab.p, d_slot_bnd.p,
                                     d_counts.p, d_sol.p, d_los.p, d_src.p, stream, &d_pipe.p[q].gate, d_csum.p,
                                     d_logn.p, zero, d_wide_ctr.p));
      phd_release(stream);
    } else {
      // the scatter reads the staging buffer in host memory directly (no copy-engine hops
      // between the wait kernel and the sweep)
      HIPCHK(launch_scatter_clusters(h_stage_buf[pre.buf].p, K, dp, d, bw, 1, d_slot_codes.p, d_slot_tab.p,
                                     d_slot_bnd.p, d_counts.p, d_sol.p, d_los.p, d_src.p, stream, &d_pipe.p[q].gate,
                                     d_csum.p, d_logn.p, zero, d_wide_ctr.p));
    }
    summary_by_scatter = true;
    pre.round_ok = launch_round(0, K, m, nullptr, track, kRoundAll, &d_pipe.p[q], q) == kOk;
    summary_by_scatter = false;
    // the staging buffer's release marker after the round, not between the scatter and the
    // round's first kernel: an event record there cost the sweep a ~6 us gap
    if (!dev) HIPCHK(hipEventRecord(ev_stage_buf[pre.buf], stream));
    stats.pipe_enqueued++;
  }
  void pre_release() {
    if (!pre.active) return;
    if (pre_dev_decision() == 1) {
      // the device gave the go for a sweep the host now drops: the chain state is no longer
      // defined (never expected: the device goes only where the host would)
      (void)hipStreamSynchronize(stream);
      have_state = false;
      err = "a sweep went ahead on the device after the host released it";
      stats.pipe_desync++;
    }
    pre.active = false;
    __atomic_store_n(&h_pipe.p[pre.par].flag, 2, __ATOMIC_RELEASE);
  }
  // Go for the sweep enqueued ahead: its draws reserved and handed over, its tables (the
  // update's held staging buffer) become the committed ones, the next speculative update
  // started.  False (nothing done) when it cannot run.
  bool pipe_go(int m) {
    // (PipeAuto: the wait kernel may have given the go itself; the host then follows it)
    const bool went = pre_dev_decision() == 1;
    const bool agree = pre.active && pre.round_ok && pre.m == m && commit_later.active && last_sweep_rounds == 1 &&
                       last_sweep_moves == 0 && !tables_dirty;
    if (went && !(agree && pre.dev && commit_later.dev && freq_dev_valid && freq_version == labels_version)) {
      (void)hipStreamSynchronize(stream);
      have_state = false;
      err = "a sweep went ahead on the device where the host would not have";
      stats.pipe_desync++;
      pre.active = false;
      return false;
    }
    if (!went) {
      if (!agree) return false;
      if (pre.dev ? (!commit_later.dev || !dspec_on()) : (commit_later.dev || commit_later.buf != pre.buf || !host_spec()))
        return false;
      if (!(freq_dev_valid && freq_version == labels_version)) return false;
      // the wait kernel gives up after pipe_limit_ticks: a go late enough to race its limit
      // is refused (the sweep is then released and prepared again); a go the kernel still
      // misses is recovered in neal8_sweep (kPipeOff)
      if (pipe_host_check &&
          std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - pre.t_enq).count() >
              (double)pipe_limit_ticks * 0.01 * 0.25) {
        stats.pipe_refused++;
        return false;
      }
    }
    rng_sync();
    const Rng saved = rng;
    const uint32_t* raw = device_draws((int64_t)n * (m + 1));
    PipeSlot& sl = h_pipe.p[pre.par];
    if (went) {
      // the draws the device chose (the same stretch of the stream, in a window it waited for)
      raw = __atomic_load_n(&sl.raw_dev, __ATOMIC_ACQUIRE);
      stats.pipe_auto++;
    } else {
      bool waited = false;
      for (int k = 0; k < 2; ++k)
        if (win[k].gen == pre.gen[k] && raw >= win[k].raw.p && raw < win[k].raw.p + win[k].count) waited = true;
      if (!waited) {                       // a window the enqueued kernels did not wait for
        pend.active = false;
        phidev.valid = false;
        rng = saved;
        return false;
      }
      __atomic_store_n(&sl.raw, raw, __ATOMIC_RELAXED);
      __atomic_store_n(&sl.flag, 1, __ATOMIC_RELEASE);
    }
    pre.active = false;
    mark("go");
    ahead.saved = saved;
    ahead.raw = raw;
    ahead.m = m;
    ahead.lv = labels_version;
    ahead.launched = true;
    ahead.prefix = false;
    ahead.track = pre.track;
    ahead.par = pre.par;
    ahead.piped = true;
    ahead.active = true;
    stats.prepass_points += n;
    stats.pipe_runs++;
    // the tables of this iteration: copied and scattered by the enqueued kernels
    commit_later.active = false;
    if (pre.dev) {
      commit_later.dev = false;
      stage_full = false;
      // the chained update enqueued behind the one just committed, else a new one; then the
      // next iteration's, chained behind it (both wait for the enqueued scatter, ev_phd_free)
      if (!dspec_promote(m)) dspec_launch();
      dnext_launch(m);
    } else {
      stage_last = pre.buf;
      stage_full = true;
      if (stage_hold == pre.buf) stage_hold = -1;
      spec_launch();
    }
    mark("ahead.spec");
    return true;
  }

  int neal8_sweep(int m) {
    // the sweep prepared at the end of the last iteration (prepare_next_sweep), if nothing
    // has changed since
    const bool use_ahead = ahead.active && ahead.m == m && ahead.lv == labels_version && !tables_dirty;
    if (!use_ahead) cancel_ahead();
    if (!have_state) { err = "no state"; return kArg; }
    if (P <= 0) { err = "no latent pool"; return kArg; }
    if (m <= 0) { err = "m must be positive"; return kArg; }
    // validate_state before the first case (the reference stops at the first point)
    {
      if (!host_c_valid || host_c_device) { /* device labels are always consistent with K */ }
      else {
        std::vector<char> seen(K + 1, 0);
        int u = 0;
        for (int i = 0; i < n; ++i) {
          const int c = h_c[i];
          if (c >= K) { cancel_ahead(); err = "State validation failed: inconsistent cluster count"; return kValidate; }
          if (!seen[c]) { seen[c] = 1; u++; }
        }
        if (u != K) { cancel_ahead(); err = "State validation failed: inconsistent cluster count"; return kValidate; }
      }
    }
    if (tables_dirty) upload_clusters();
    // update_phi can be speculated during the sweep when the host holds the pre-sweep
    // frequency tables of every label and the sweep carries them (move log)
    const bool spec_go = freq_dev_valid && freq_version == labels_version && !(debug & 128) && !recount_only() &&
                         host_spec();
    const bool freq_before_ok = freq_version == labels_version && !recount_only();
    // or on the device beside the sweep (phi_mode 1)
    const bool dspec_go = freq_dev_valid && freq_version == labels_version && !recount_only() && dspec_on();
    if (!use_ahead) {
      spec.ran = false;
      dspec.ran = false;
    }
    spec.lv = 0;
    labels_version++;
    const int K0 = K;
    int sweep_moves = 0;
    const bool hc_before = host_c_valid;     // the host label mirror before the sweep
    std::vector<uint8_t> old_center = h_center;
    std::vector<double> old_sigma = h_sigma;

    // the sweep's slice of the R stream (m pick uniforms + 1 categorical per point),
    // generated on the device; the host stream continues after it
    auto tr0 = std::chrono::steady_clock::now();
    const size_t nraw = (size_t)n * (m + 1);
    const uint32_t* d_sweep_raw = use_ahead ? ahead.raw : device_draws((int64_t)nraw);
    const bool ahead_launched = use_ahead && ahead.launched;
    const bool ahead_prefix = use_ahead && ahead.prefix && !ahead.launched;
    const bool ahead_piped = ahead_launched && ahead.piped;
    if (ahead_launched || ahead_prefix) par = ahead.par;
    else par ^= 1;
    ahead.active = false;
    mark("draws");
    // update_phi speculated on the pool while this thread launches the sweep
    struct SpecGuard {
      Ctx* c;
      ~SpecGuard() {
        if (c->spec.ran && !c->spec.joined && c->pj_open) {   // not joined (early exit)
          (void)c->pj_finish();
          c->spec.ran = false;
        }
      }
    } spec_guard{this};
    if (spec_go && !use_ahead) spec_launch();
    else if (dspec_go && !use_ahead) dspec_launch();
    stats.t_rng_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr0).count();

    int nslots = K;
    int p = 0;
    bool end_queued = false;             // the sweep end is on the stream behind the last launch
    const int64_t rounds0 = stats.rounds;
    // round 0 may already be on the device (prepare_next_sweep with launch)
    const bool launched_ahead = ahead_launched;
    const bool track = (launched_ahead || ahead_prefix) ? ahead.track : (freq_dev_valid && !recount_only());
    if (!launched_ahead && !ahead_prefix) sweep_buffers(track, m);
    while (p < n) {
      if (!(launched_ahead && stats.rounds == rounds0)) {
        // round 0 after a prepared prefix: the resolver part only (same arguments)
        const int part = (ahead_prefix && stats.rounds == rounds0) ? kRoundResolve : kRoundAll;
        const int lst = launch_round(p, nslots, m, d_sweep_raw, track, part);
        if (lst) return lst;
        // while sweeps keep moving points, the sweep-end kernels go behind every launch at
        // once (they act only after the launch that completes the sweep): no host round trip
        // between the resolver and the sweep end
        end_queued = last_sweep_moves > 0;
        if (end_queued) launch_sweep_end(scap - 2, track);
      } else {
        end_queued = false;
      }
      mark("launched");
      if (stats.rounds == rounds0) {   // hidden behind the device work
        // (not while sweeps keep moving points: the enqueued sweep would be dropped)
        if (deep_ok && (host_spec() ? (spec.ran && spec.K == K) : (dspec.ran && dspec.K == K)) && track &&
            last_sweep_moves == 0 && !(debug & 4194304)) {
          pre_enqueue(m, track);
          mark("pre");
        }
        if (spec.ran) spec_join();
        else if (host_spec()) prefill_phi_stream();
      }
      mark("prefill");
      HIPCHK(hipEventSynchronize(ev_res[par]));
      mark("resolved");
      const bool piped_round = ahead_piped && stats.rounds == rounds0;
      if (piped_round ? pre_timed[par] : round_timed) {
        float t1 = 0;
        if (piped_round) round_points = n;
        HIPCHK(hipEventElapsedTime(&t1, piped_round ? ev_pp[par][0] : ev[0], piped_round ? ev_pp[par][1] : ev[1]));
        stats.t_prepass_ms += t1;
        stats.prepass_timed++;
        stats.prepass_timed_points += round_points;
      }
      if (round_fine && !piped_round) {
        float t2 = 0, t3 = 0;
        HIPCHK(hipEventElapsedTime(&t3, ev[1], ev[5]));
        HIPCHK(hipEventElapsedTime(&t2, ev[5], ev[2]));
        stats.t_exact_ms += t3;
        stats.t_resolve_ms += t2;
      }
      stats.rounds++;
      const ResolveCtl c = *ctl_at(par);
      if (c.status == kPipeOff && piped_round) {
        // the sweep enqueued ahead was gated off on the device (its wait kernel's limit
        // passed before the host's go reached it): none of its kernels ran, the tables of
        // this iteration (the held staging buffer) were not scattered and round 0's
        // k_cluster_summary did not clear the move count.  Commit the tables and run the
        // sweep ungated from point 0 with the same draws.
        if (pre.dev || stage_last < 0 || !stage_full) {
          upload_clusters();               // from the host's parameters (the device update's)
        } else {
          stage_fill = stage_last;
          stage_commit(upload_layout(K, dp, d, bw), K, true);
        }
        if (track) mcount_clear = true;
        stats.pipe_recovered++;
        continue;
      }
      // the sweep enqueued ahead runs only after a complete sweep without moves
      if (pre.active && (c.status || c.next < n || c.moves)) pre_release();
      last_sweep_rounds = (int)(stats.rounds - rounds0);
      if ((debug & 2) && last_fp && last_fpg) {
        long long tp[16];
        HIPCHK(hipMemcpy(tp, d_rprof.p, sizeof(tp), hipMemcpyDeviceToHost));
        std::fprintf(stderr,
                     "[resolve_fpg] G %d: %lld listed in %lld windows, %lld rounds; init %.2f us, rounds %.2f us, drift / "
                     "re-test / commit %.2f us, in grid barriers %.2f us, total %.2f us\n",
                     last_fpg, tp[9], tp[8], tp[5], (tp[1] - tp[0]) / 100.0, tp[3] / 100.0, tp[4] / 100.0, tp[2] / 100.0,
                     (tp[7] - tp[0]) / 100.0);
      } else if ((debug & 2) && last_fp) {
        long long tp[16];
        HIPCHK(hipMemcpy(tp, d_rprof.p, sizeof(tp), hipMemcpyDeviceToHost));
        std::fprintf(stderr,
                     "[resolve_fp] init %.2f us, %lld listed in %lld chunks: rounds %lld (%.2f us), drift / re-test / "
                     "commit %.2f us, %lld stops (%.2f us), total %.2f us; in rounds: counts %.2f us, ballots %.2f us, "
                     "evaluations (slowest wave) %.2f us, %lld evaluations, %lld own draws (row loads + draws: %.2f us, summed over waves)\n",
                     (tp[1] - tp[0]) / 100.0, tp[9], tp[8], tp[5], tp[3] / 100.0, tp[4] / 100.0, tp[6], tp[2] / 100.0,
                     (tp[7] - tp[0]) / 100.0, tp[10] / 100.0, tp[11] / 100.0, tp[12] / 100.0, tp[14], tp[15], tp[13] / 100.0);
      } else if (debug & 2) {
        long long tp[16];
        HIPCHK(hipMemcpy(tp, d_rprof.p, sizeof(tp), hipMemcpyDeviceToHost));
        std::fprintf(stderr,
                     "[resolve] init %.2f us, batches %.2f us, decided points %lld in %.2f us (exact decisions "
                     "%.2f us, state updates %.2f us, re-tests %.2f us over %lld points; block mode: %lld blocks), "
                     "total %.2f us\n",
                     (tp[1] - tp[0]) / 100.0, tp[3] / 100.0, tp[6], tp[4] / 100.0, tp[12] / 100.0, tp[14] / 100.0,
                     tp[13] / 100.0, tp[15], tp[5], (tp[7] - tp[0]) / 100.0);
      }
      stats.exact_points += c.exact;
      stats.listed_points += c.listed;
      last_exact = c.exact;
      last_listed = c.listed;
      // a sweep's first launch sets the density (a restart's tail of the sweep is not typical)
      // (a dense launch listed every point: its density is what the prepass's margin test
      // would have listed, counted by k_snap_draws)
      if (p == 0 || last_density < 0)
        last_density = (double)(c.uncertain >= 0 ? c.uncertain : c.listed) / (double)std::max(1, n - p);
      stats.moves += c.moves;
      sweep_moves += c.moves;
      stats.checked_rounds += c.checked;
      last_unsettled = c.checked || (c.restart && c.next < n);
      if (c.aborted && !c.status) {
        // k_resolve_fpg gave up at a grid barrier (a workgroup not resident within the limit):
        // everything before c.next is committed; the restart runs on one workgroup
        stats.fpg_aborts++;
        fpg_skip = true;
      }
      if (c.status) {
        err = c.status == kValidate ? "State validation failed: inconsistent cluster count from Neal8 case 2"
              : c.status == kWalker ? "Walker alias table failure"
              : c.status == kProb   ? "Too few positive probabilities"
              : c.status == kPipeOff ? "a sweep enqueued ahead was gated off on the device"
                                    : "resolver failure";
        if (c.status == kPipeOff) return kArg;
        return c.status;
      }
      K = c.K;
      nslots = c.nslots;
      if (c.restart) stats.restarts++;
      p = c.next;
    }

    // slots -> labels; rebuild per-label parameters and counts from the resolver summary
    auto ts0 = std::chrono::steady_clock::now();
    const int* sol = (const int*)ctl_at(par) + kCtlInts;
    const int* cnt = sol + scap;
    const int* src = cnt + scap;
    if (sweep_moves > 0) {
      if (!end_queued) launch_sweep_end(nslots, track);
      if (track) {   // the gather wrote freq2 (and its copy is on its way)
        std::swap(d_freq.p, d_freq2.p);
        std::swap(d_freq.n, d_freq2.n);
        freq_d2h_version = labels_version;
        freq_next_pending = true;    // into h_freq_next; update_phi swaps it in
      } else {
        freq_dev_valid = false;      // not carried: the next update_phi recounts
      }
    } else if (track && freq_before_ok) {
      // nothing moved: the host's tables are still current
      freq_version = labels_version;
      freq_d2h_version = labels_version;
      freq_next_pending = false;
    }
    h_center.assign((size_t)K * d, 0);
    h_sigma.assign((size_t)K * d, 0.0);
    h_counts.assign(K, 0);
    bool fetched = false;
    for (int l = 0; l < K; ++l) {
      const int s = sol[l];
      h_counts[l] = cnt[s];
      if (s < K0) {
        std::memcpy(&h_center[(size_t)l * d], &old_center[(size_t)s * d], d);
        std::memcpy(&h_sigma[(size_t)l * d], &old_sigma[(size_t)s * d], (size_t)d * 8);
      } else {
        pool_entry(src[s], &h_center[(size_t)l * d], &h_sigma[(size_t)l * d]);
        fetched = true;
      }
    }
    if (fetched && pool_on_device) HIPCHK(hipStreamSynchronize(stream));
    // the host's label mirror: a sweep without moves changes no label; with moves, and the
    // labels still in slot order (same K, every label on its own slot), the move log gives the
    // new labels of the moved points (12 B each: the recording path's labels without an N-word
    // download, mirror_moves); anything else invalidates the mirror
    mirror_moves = 0;
    if (!hc_before || sweep_moves > 0) host_c_valid = false;
    // (a mirror kept across the sweep now mirrors device labels: consistent with K by
    // construction, so the next sweep does not re-validate it over N points)
    if (host_c_valid) host_c_device = true;
    if (hc_before && sweep_moves > 0 && track && K == K0 && sweep_moves <= n / 16) {
      bool ident = true;
      for (int l = 0; l < K && ident; ++l) ident = sol[l] == l;
      if (ident) mirror_moves = sweep_moves;
    }
    tables_dirty = true;
    if (dspec.ran) {
      dspec.lv = labels_version;
      dspec.moves = sweep_moves;
    }
    if (spec.ran) {
      // leading labels with the same slot (hence parameters) and count as at the speculation
      spec.lv = labels_version;
      spec.moves = sweep_moves;
      int pfx = 0;
      while (pfx < std::min(K, spec.K) && sol[pfx] == pfx && h_counts[pfx] == spec.counts[pfx]) ++pfx;
      spec.pfx = pfx;
    }
    last_sweep_moves = sweep_moves;
    mark("sweep_end");
    stats.t_stats_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts0).count();
    stats.sweeps++;
    return kOk;
  }

  // ------------------------------------------------------------------ update_phi
  // freq[k][j][l] for the labels in mask (device histogram), downloaded to h_freq.
  void histogram(const std::vector<unsigned char>* mask) {
    histogram_launch(mask);
    histogram_wait(mask);
  }
  void histogram_launch(const std::vector<unsigned char>* mask) {
    const size_t nent = (size_t)K * d * mmax;
    h_freq.ensure(std::max<size_t>(nent, 1));
    if (!mask && freq_dev_valid && !recount_only()) {
      // the per-label tables were carried through the sweep by the move log (and usually
      // copied out behind it already)
      if (freq_d2h_version != labels_version) {
        HIPCHK(hipMemcpyAsync(h_freq.p, d_freq.p, nent * 4, hipMemcpyDeviceToHost, stream));
        freq_next_pending = false;
      }
      return;
    }
    DevBuf<unsigned>& dst = mask ? d_freq_m : d_freq;
    if (mask) dst.ensure(std::max<size_t>(nent, 1));
    else ensure_slots(K + 2);
    HistArgs ha;
    ha.codes_t = d_codes_t.p; ha.n = n; ha.d = d; ha.nq = nq; ha.label = d_c.p;
    ha.mask = nullptr; ha.K = K; ha.mmax = mmax; ha.freq = dst.p;
    ha.xpk = d_xpk.p; ha.W = W; ha.wb = wb;
    {
      int nbx, kc, tpb;
      const size_t pw = hist_partial_words(ha, &nbx, &kc, &tpb);
      d_hist_part.ensure(std::max<size_t>(pw, 1));
      ha.partial = pw ? d_hist_part.p : nullptr;
    }
    if (mask) {
      d_mask.ensure(std::max(K, 1));
      h_mask.ensure(std::max(K, 1));
      std::memcpy(h_mask.p, mask->data(), K);
      HIPCHK(hipMemcpyAsync(d_mask.p, h_mask.p, K, hipMemcpyHostToDevice, stream));
      ha.mask = d_mask.p;
    }
    HIPCHK(launch_hist(ha, stream));
    if (!mask) {
      freq_dev_valid = true;
      freq_next_pending = false;
    }
    HIPCHK(hipMemcpyAsync(h_freq.p, dst.p, nent * 4, hipMemcpyDeviceToHost, stream));
  }
  void histogram_wait(const std::vector<unsigned char>* mask) {
    HIPCHK(hipStreamSynchronize(stream));
    freq_version = mask ? 0 : labels_version;
  }

  struct PhiItem {
    int err, lstar;
    int mode;                // sample_prob1_prep: 0 cumulative, 1 Walker alias table
    bool bp;                 // rhig beta path for lstar
    RBeta rb;                // rbeta(w + 1, v - 1) setup for lstar
    // phase B -> C
    int path;                // 1 beta, 2 bisection
    double x, nv, nw;        // beta draw x or Omega; sigma parameters of the drawn center
  };
  std::vector<PhiItem> phi_items;
  std::vector<double> phi_cum;
  std::vector<int> phi_perm, phi_off;

  // Speculative update_phi.  A Neal-8 sweep consumes exactly N (m + 1) uniforms whatever it
  // decides, so the stream position of the update_phi that follows is known before the
  // sweep runs, and update_phi of a cluster depends only on that cluster's size, frequency
  // table and parameters.  While the device sweeps, the host runs update_phi on the
  // pre-sweep state (spec_launch / spec_join); afterwards the results of the leading clusters the
  // sweep left untouched (same slot, same count, same frequency table) are exactly
  // update_phi's, and the draws resume from the stream offset where the first touched
  // cluster's began.  A sweep without moves leaves every cluster untouched: update_phi is
  // then done before the device finishes.
  struct PhiSpec {
    bool ran = false;
    bool joined = false;               // spec_join collected the job
    uint64_t lv = 0;                   // labels_version the results apply to (set at the sweep end)
    uint64_t pos = 0, epoch = 0;       // stream position of the first draw
    int K = 0;                         // labels at the speculation
    int nvalid = 0;                    // clusters 0..nvalid-1 complete (no error, inside the prefetched stream)
    int moves = -1;                    // reassignments of the sweep (set at its end)
    int pfx = 0;                       // leading labels whose slot and count the sweep kept
    std::vector<uint8_t> center;
    std::vector<double> sigma;
    std::vector<int> counts;
    std::vector<int64_t> off;          // stream offset at the start of cluster t's draws
    int stage_buf = -1;                // staging buffer of its tables (stage_hold until used)
  } spec;
  Rng spec_live;                       // spill target of the speculative pass (never the chain's)
  PinBuf<unsigned> h_freq_next;        // the sweep's frequency copy-out (h_freq keeps the pre-sweep one)
  bool freq_next_pending = false;

  // phi_stream from the chain's current state (after rng_sync): from the copy of the
  // device window when it holds the slice, else generated here.  False if never seeded.
  bool fill_phi_stream(int64_t N) {
    StreamAhead& sa = phi_stream;
    bool dev = phidev.valid && phidev.pos == rng.pos && phidev.epoch == rng.epoch && phidev.mti == rng.mti &&
               phidev.N == N;
    if (dev) {
      HIPCHK(hipEventSynchronize(phidev.ev));
      if (pj_open) pj.ns_f2.store(pj_ns());
      for (int i = 0; i < 624 && dev; ++i) dev = mt_untemper(phidev.blk[i]) == rng.mt[i];
    }
    if (dev) {
      sa.fill_raw(rng, phidev.blk, phidev.N);
      return true;
    }
    return sa.fill(rng, N);
  }

  // A slice of N uniforms for the split-merge update_phi jobs: the device window's words
  // when the last device_draws prefetched at least N of them from this position (the
  // scan's draws came from a window), else generated on the host.
  bool fill_stream_from(int64_t N) {
    StreamAhead& sa = phi_stream;
    bool dev = phidev.valid && phidev.pos == rng.pos && phidev.epoch == rng.epoch && phidev.mti == rng.mti &&
               phidev.N >= N;
    if (dev) {
      HIPCHK(hipEventSynchronize(phidev.ev));
      for (int i = 0; i < 624 && dev; ++i) dev = mt_untemper(phidev.blk[i]) == rng.mt[i];
    }
    if (dev) {
      sa.fill_raw(rng, phidev.blk, N);
      return true;
    }
    return sa.fill(rng, N);
  }

  // update_phi's slice of the host stream, generated ahead (also called while the device
  // runs a sweep, which draws only from the device windows).
  void prefill_phi_stream() {
    HostPool::get().prewake();        // for the logits below, then update_phi's phases
    rng_sync();
    StreamAhead& sa = phi_stream;
    if (sa.n > 0 && sa.used == 0 && sa.start.pos == rng.pos && sa.start.epoch == rng.epoch) return;
    if (fill_phi_stream(phi_prefetch)) {
      sa.used = 0;
      HostPool::get().run(sa.n, 1024, [&](int64_t a0, int64_t a1) { sa.logits(a0, a1); });
      sa.avail = INT64_MAX;
    }
  }

  void stage_entry_from(const UploadLayout& L, int r, int k, const uint8_t* cen, const double* sig, int count) {
    uint8_t* st = h_stage_buf[pj.stage_buf].p;
    double* tt = (double*)(st + L.off_tab) + (size_t)r * 2 * d;
    tables_for(cen, sig, st + L.off_codes + (size_t)r * dp, tt);
    bounds_for(cen, tt, (uint64_t*)(st + L.off_bnd) + (size_t)r * bw);
    ((int*)(st + L.off_counts))[r] = count;
    ((int*)(st + L.off_slot))[r] = k;
  }

  // cf:511-591 as a pool job over the clusters touched[t0..T), with cluster sizes `counts`,
  // frequencies `freq` (freq[k][j][level]) and current sigma from h_sigma, drawing from
  // phi_stream.  The new centers / sigmas go to Cen / Sig (label-indexed), the label tables
  // to the staging buffer L (entry k when `full`, else t).  Phases:
  //   fill (one task)  the stream slice (phi_stream), when the job generates it;
  //   logits           log(u / (1 - u)) and log(u u u') of the slice, in chunks;
  //   A (parallel)     per (cluster, attribute): center probabilities (cf:537-556), Rcpp
  //                    sample's FixupProb / revsort / cumulative sums, and the rhig branch and
  //                    rbeta setup for the most probable center;
  //   B (one thread)   the reference's draw order: per cluster, its d center uniforms, then
  //                    its d sigma draws (rbeta rejection loops, or the bisection's Omega);
  //   C (parallel)     sigma = -1/log(out) and the bisection solves, then the label tables.
  // Every value is computed by the same expressions as the one-pass loop, so the chain is
  // unchanged.  Tasks are handed out through shared counters; every thread (the caller
  // too) takes what is ready, and a thread waiting on a dependency runs that dependency's
  // tasks itself, so the job completes whichever threads the OS runs.
  struct PhiJob {
    std::vector<int> touched;
    int t0 = 0, T = 0, nach = 1, achunk = 1, sumatt = 0;
    const int* counts = nullptr;
    const unsigned* freq = nullptr;
    uint8_t* Cen = nullptr;
    double* Sig = nullptr;
    UploadLayout L{};
    bool full = false;
    int64_t* offs = nullptr;           // offs[t]: stream offset at the start of cluster t's draws
    bool spec = false;                 // speculative: the slice is generated by the job from rng
    int64_t fill_count = 0;
    // logit chunks: small first ones (B starts on the first as soon as it is done), then
    // 1024 entries
    static constexpr int kLogitChunk = 1024, kSmall = 128, kNSmall = 8;
    static int64_t chunk_beg(int c) {
      return c <= kNSmall ? (int64_t)c * kSmall : (int64_t)kNSmall * kSmall + (int64_t)(c - kNSmall) * kLogitChunk;
    }
    static int chunk_of(int64_t pos) {
      return pos < kNSmall * kSmall ? (int)(pos / kSmall) : kNSmall + (int)((pos - kNSmall * kSmall) / kLogitChunk);
    }
    std::atomic<int> fill{0};          // 0 open, 1 taken, 2 done
    std::atomic<int> nextL{0}, doneL{0};
    std::atomic<int> nL{0};
    std::unique_ptr<std::atomic<uint8_t>[]> ldone;   // per logit chunk: computed
    int ldone_cap = 0;
    std::atomic<int> nextA{0};
    std::unique_ptr<std::atomic<int>[]> stA, stB;
    std::atomic<int> bclaim{0};
    std::atomic<int> nextC{0}, gsl{-1};
    int berr = 0, b_end = 0;
    bool failed = false;
    int stage_buf = 0;                 // staging buffer phase C fills
    const double* sig_in = nullptr;    // current sigmas (phase A), indexed like Sig
    bool stage = true;                 // phase C stages the label tables into L
    // diagnostics (debug bit 5): ns after launch
    std::chrono::steady_clock::time_point t_launch;
    std::atomic<int64_t> ns_fill{0}, ns_logits{0}, ns_b0{0}, ns_b1{0}, ns_f0{0}, ns_f1{0}, ns_f2{0};
    int64_t ns_wait_a = 0, ns_wait_l = 0;   // (debug bit 5) B's waits for phase A / logit chunks
    int64_t b_draws = 0, b_clusters_extra = 0;   // (debug bit 5) B's draws, clusters with an extra draw
    std::atomic<int> b_thread{0};
  } pj;
  int64_t pj_ns() const {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - pj.t_launch).count();
  }
  void tsum(const char* name, double us) {
    trace_add(name, us);
  }

  void pj_phaseA(int t, int j0, int j1) {
    const int k = pj.touched[t];
    const int nn = pj.counts[k];
    for (int j = j0; j < j1; ++j) {
      const int mj = att[j];
      const unsigned* fj = &pj.freq[((size_t)k * d + j) * mmax];
      const double sg = pj.sig_in[(size_t)k * d + j];
      double prob[256];
      for (int l = 0; l < mj; ++l) prob[l] = (-((double)nn - (double)fj[l])) / sg;
      double mx = prob[0];
      for (int l = 1; l < mj; ++l) if (prob[l] > mx) mx = prob[l];
      for (int l = 0; l < mj; ++l) prob[l] = std::exp(prob[l] - mx);
      double sum = 0.0;
      for (int l = 0; l < mj; ++l) sum += prob[l];
      for (int l = 0; l < mj; ++l) prob[l] = prob[l] / sum;
      PhiItem& P = phi_items[(size_t)t * d + j];
      double* cum = &phi_cum[(size_t)t * pj.sumatt + phi_off[j]];
      int* perm = &phi_perm[(size_t)t * pj.sumatt + phi_off[j]];
      const int mode = sample_prob1_prep(prob, mj, cum, perm);
      P.err = mode < 0 ? -mode : 0;
      P.mode = mode;
      P.lstar = -1;
      if (P.err || mode == 1) continue;       // no likely center to speculate on (Walker)
      const int l = perm[0] - 1;
      const double sumdelta = (double)fj[l];
      const double nw_ = w[j] + nn - sumdelta, nv_ = v[j] + sumdelta;
      P.lstar = l;
      P.bp = rhig_beta_path(nv_, nw_, (double)mj);
      if (P.bp) P.rb = rbeta_setup(nw_ + 1, nv_ - 1);
    }
  }

  // the stream-consuming draws of cluster t (reference order)
  int pj_phaseB(int t) {
    StreamAhead& sa = phi_stream;
    const int k = pj.touched[t];
    const int nn = pj.counts[k];
    const unsigned* freq = pj.freq;
    const int sumatt = pj.sumatt;
    uint8_t* cen = &pj.Cen[(size_t)k * d];
    // the items were written by other cores: prefetch a few ahead (cross-core misses
    // would otherwise serialise this loop)
    constexpr int kAhead = 8;
    for (int j = 0; j < std::min(d, kAhead); ++j) {
      __builtin_prefetch(&phi_items[(size_t)t * d + j]);
      __builtin_prefetch(&phi_cum[(size_t)t * sumatt + phi_off[j]]);
    }
    for (int j = 0; j < d; ++j) {
      if (j + kAhead < d) {
        const size_t ja = (size_t)t * d + j + kAhead;
        __builtin_prefetch(&phi_items[ja]);
        __builtin_prefetch((const char*)&phi_items[ja] + 64);
        __builtin_prefetch(&phi_cum[(size_t)t * sumatt + phi_off[j + kAhead]]);
        __builtin_prefetch(&phi_perm[(size_t)t * sumatt + phi_off[j + kAhead]]);
        __builtin_prefetch(&freq[((size_t)k * d + j + kAhead) * mmax]);
      }
      const PhiItem& P = phi_items[(size_t)t * d + j];
      if (P.err) return P.err;
      const size_t o = (size_t)t * sumatt + phi_off[j];
      cen[j] = (uint8_t)(sample_prob1_pick(&phi_cum[o], &phi_perm[o], att[j], sa.next(nullptr), P.mode) + 1);
    }
    // sigma draws.  Items go in batches of up to kSpec whose first rbeta attempts are
    // evaluated together at the stream positions they have if every earlier item of the
    // batch is accepted on its first attempt (independent work the core overlaps); they are
    // committed in order up to the first item that was not, which is then drawn
    // sequentially from its true position.  Same arithmetic either way.
    constexpr int kSpec = HDPM_PHI_SPEC;
    auto params = [&](int j, bool* bp, RBeta* rb) {
      PhiItem& P = phi_items[(size_t)t * d + j];
      const int l = cen[j] - 1;
      const double mj = (double)att[j];
      const double sumdelta = (double)freq[((size_t)k * d + j) * mmax + l];
      P.nw = w[j] + nn - sumdelta;
      P.nv = v[j] + sumdelta;
      if (l == P.lstar) {
        *bp = P.bp;
        if (*bp) *rb = P.rb;
      } else {
        *bp = rhig_beta_path(P.nv, P.nw, mj);
        if (*bp) *rb = rbeta_setup(P.nw + 1, P.nv - 1);
      }
    };
    auto sequential = [&](int j, bool bp, const RBeta& rb) {
      PhiItem& P = phi_items[(size_t)t * d + j];
      const double mj = (double)att[j];
      if (bp) {                                   // hg:359-363
        double x = rbeta_draw_s(sa, rb);
        while (x > (mj - 1) / mj) x = rbeta_draw_s(sa, rb);
        P.path = 1;
        P.x = x;
      } else {                                    // hg:365-367
        P.path = 2;
        P.x = sa.next(nullptr);
      }
    };
    int j = 0;
    while (j < d) {
      bool bps[kSpec];
      RBeta rbs[kSpec];
      int cons[kSpec];
      int nb = 0;
      int64_t q = sa.used;
      for (; nb < kSpec && j + nb < d; ++nb) {
        params(j + nb, &bps[nb], &rbs[nb]);
        cons[nb] = !bps[nb] ? 1 : rbs[nb].kind == RBeta::kBB ? 2 : 0;
        if (cons[nb] == 0 || sa.spilled || q + cons[nb] > sa.n) break;
        q += cons[nb];
      }
      const int nspec = nb;   // items with a speculative first attempt
      double xs[kSpec];
      bool ok[kSpec];
      q = sa.used;
      if (nspec > 0) sa.need(q + 2 * kSpec);
      for (int b = 0; b < nspec; ++b) {
        const double mj = (double)att[j + b];
        if (bps[b]) {
          double wv;
          ok[b] = rbeta_bb_attempt(rbs[b], sa.u[q], sa.lg[q], sa.u[q + 1], sa.lz[q], &wv);
          xs[b] = rbeta_bb_value(rbs[b], wv);
          ok[b] = ok[b] && !(xs[b] > (mj - 1) / mj);
        } else {
          xs[b] = sa.u[q];
          ok[b] = true;
        }
        q += cons[b];
      }
      int b = 0;
      for (; b < nspec && ok[b]; ++b) {
        PhiItem& P = phi_items[(size_t)t * d + j + b];
        P.path = bps[b] ? 1 : 2;
        P.x = xs[b];
        sa.used += cons[b];
      }
      j += b;
      if (j >= d) break;
      if (b < nb) {                               // item j was prepared (speculated or not)
        sequential(j, bps[b], rbs[b]);
      } else {                                    // batch ended before item j was prepared
        bool bp;
        RBeta rb;
        params(j, &bp, &rb);
        sequential(j, bp, rb);
      }
      ++j;
    }
    return 0;
  }

  // sigma of cluster t, then its staged tables; false on a GSL error
  bool pj_phaseC(int t) {
    const int k = pj.touched[t];
    bool ok = true;
    for (int j = 0; j < d; ++j) {
      PhiItem& P = phi_items[(size_t)t * d + j];
      const double mj = (double)att[j];
      double out;
      if (P.path == 1) {
        out = P.x / ((mj - 1) * (1 - P.x));
      } else {
        int e = kOk;
        out = bisec_hyper2(P.nw, P.nv, mj, P.x, &e, hig_log);
        if (e) { ok = false; continue; }
      }
      pj.Sig[(size_t)k * d + j] = -1 / std::log(out);
    }
    if (ok && pj.stage)
      stage_entry_from(pj.L, pj.full ? k : t, k, &pj.Cen[(size_t)k * d], &pj.Sig[(size_t)k * d], pj.counts[k]);
    return ok;
  }

  // Prepares pj for touched[t0..T).  With `spec`, the job itself generates the stream slice
  // (waiting for the device state first) into phi_stream, with spec_live as spill target.
  void pj_setup(std::vector<int> touched, int t0, const int* counts, const unsigned* freq, uint8_t* Cen, double* Sig,
                const UploadLayout& L, bool full, int64_t* offs, bool spec) {
    pj.touched = std::move(touched);
    pj.T = (int)pj.touched.size();
    pj.t0 = t0;
    pj.counts = counts;
    pj.freq = freq;
    pj.Cen = Cen;
    pj.Sig = Sig;
    pj.L = L;
    pj.full = full;
    pj.offs = offs;
    pj.spec = spec;
    pj.sig_in = h_sigma.data();
    pj.stage = true;
    pj.stage_buf = stage_fill;
    pj.fill_count = phi_prefetch;
    phi_off.resize(d + 1);
    phi_off[0] = 0;
    for (int j = 0; j < d; ++j) phi_off[j + 1] = phi_off[j] + att[j];
    pj.sumatt = phi_off[d];
    phi_items.resize((size_t)pj.T * d);
    phi_cum.resize((size_t)pj.T * pj.sumatt);
    phi_perm.resize((size_t)pj.T * pj.sumatt);
    // A in chunks of attributes so the first cluster is ready early
    pj.achunk = std::max(4, (d + 15) / 16);
    pj.nach = (d + pj.achunk - 1) / pj.achunk;
    pj.stA.reset(new std::atomic<int>[std::max(pj.T, 1)]);
    pj.stB.reset(new std::atomic<int>[std::max(pj.T, 1)]);
    for (int t = 0; t < pj.T; ++t) { pj.stA[t].store(0); pj.stB[t].store(0); }
    pj.fill.store(spec ? 0 : 2);
    if (!spec) phi_stream.avail = INT64_MAX;     // filled and logits computed beforehand
    pj.nL.store(0);
    pj.nextL.store(0);
    pj.doneL.store(0);
    pj.nextA.store(t0 * pj.nach);
    pj.bclaim.store(t0 >= pj.T ? 1 : 0);
    pj.nextC.store(t0);
    pj.gsl.store(-1);
    pj.berr = 0;
    pj.b_end = t0;
    pj.failed = false;
    if (offs && t0 >= pj.T) offs[pj.T] = phi_stream.used;
  }

  bool pj_fill() {
    int z = 0;
    if (pj.fill.load(std::memory_order_acquire) != 0 || !pj.fill.compare_exchange_strong(z, 1)) return false;
    StreamAhead& sa = phi_stream;
    try {
      pj.ns_f0.store(pj_ns());
      rng_sync();                               // the device state at the sweep's end
      pj.ns_f1.store(pj_ns());
      spec_live = rng;
      if (!fill_phi_stream(pj.fill_count)) sa.n = 0;
    } catch (const HipError&) {                 // the caller meets the error again; no speculation
      sa.n = 0;
      pj.failed = true;
    }
    sa.used = 0;
    sa.live = &spec_live;
    const int nl = sa.n > 0 ? PhiJob::chunk_of(sa.n - 1) + 1 : 0;
    if (nl > pj.ldone_cap) {
      pj.ldone.reset(new std::atomic<uint8_t>[nl]);
      pj.ldone_cap = nl;
    }
    for (int c = 0; c < nl; ++c) pj.ldone[c].store(0, std::memory_order_relaxed);
    // B may start on the first chunks: later positions wait for (or compute) their chunk
    sa.avail = 0;
    sa.wait_avail = [this](int64_t pos) { return pj_wait_chunk(pos); };
    pj.nL.store(nl, std::memory_order_relaxed);
    pj.ns_fill.store(pj_ns());
    pj.fill.store(2, std::memory_order_release);
    return true;
  }
  // limit: only chunks below it (the first ones, before phase A's first clusters)
  bool pj_logit(int limit = INT_MAX) {
    if (pj.fill.load(std::memory_order_acquire) != 2) return false;
    if (pj.nextL.load(std::memory_order_relaxed) >= limit) return false;
    const int c = pj.nextL.fetch_add(1);
    if (c >= pj.nL.load(std::memory_order_relaxed)) return false;
    StreamAhead& sa = phi_stream;
    sa.logits(PhiJob::chunk_beg(c), std::min<int64_t>(sa.n, PhiJob::chunk_beg(c + 1)));
    pj.ldone[c].store(1, std::memory_order_release);
    if (pj.doneL.fetch_add(1, std::memory_order_release) + 1 == pj.nL.load()) pj.ns_logits.store(pj_ns());
    return true;
  }
  // B's reads at `pos`: wait for its logit chunk (computing chunks meanwhile); returns the
  // end of the leading run of computed chunks
  int64_t pj_wait_chunk(int64_t pos) {
    const StreamAhead& sa = phi_stream;
    const int nl = pj.nL.load(std::memory_order_relaxed);
    int c = PhiJob::chunk_of(pos);
    if (c >= nl) return INT64_MAX;
    if (!pj.ldone[c].load(std::memory_order_acquire)) {
      const int64_t w0 = (debug & 32) ? pj_ns() : 0;
      while (!pj.ldone[c].load(std::memory_order_acquire))
        if (!pj_logit()) HostPool::spin_pause();
      if (debug & 32) pj.ns_wait_l += pj_ns() - w0;
    }
    while (c + 1 < nl && pj.ldone[c + 1].load(std::memory_order_acquire)) ++c;
    return c + 1 >= nl ? INT64_MAX : std::min<int64_t>(sa.n, PhiJob::chunk_beg(c + 1));
  }
  // limit: only tasks of clusters below it
  bool pj_take_a(int limit = INT_MAX) {
    if (limit < pj.T && pj.nextA.load(std::memory_order_relaxed) >= limit * pj.nach) return false;
    const int task = pj.nextA.fetch_add(1);
    if (task >= pj.T * pj.nach) return false;
    const int t = task / pj.nach, c = task - t * pj.nach;
    pj_phaseA(t, c * pj.achunk, std::min(d, (c + 1) * pj.achunk));
    pj.stA[t].fetch_add(1, std::memory_order_acq_rel);
    return true;
  }
  bool pj_stream_ready() const {
    if (pj.fill.load(std::memory_order_acquire) != 2) return false;
    const int nl = pj.nL.load(std::memory_order_relaxed);
    if (debug & 4096) return pj.doneL.load(std::memory_order_acquire) >= nl;   // all logits first
    return nl == 0 || pj.ldone[0].load(std::memory_order_acquire);
  }
  // B for every cluster, in order, on the thread that claims it once the stream is ready
  bool pj_try_b() {
    int z = 0;
    if (pj.bclaim.load(std::memory_order_acquire) != 0 || !pj_stream_ready() || !pj.bclaim.compare_exchange_strong(z, 1))
      return false;
    StreamAhead& sa = phi_stream;
    pj.ns_b0.store(pj_ns());
    pj.b_thread.store(sched_getcpu() == HostPool::get().main_cpu() ? 1 : 0);
    int tb = pj.t0;
    pj.ns_wait_a = pj.ns_wait_l = 0;
    pj.b_draws = 0;
    pj.b_clusters_extra = 0;
    const int64_t used0 = sa.used;
    for (; tb < pj.T; ++tb) {
      const int64_t u0 = sa.used;
      if (pj.stA[tb].load(std::memory_order_acquire) < pj.nach) {
        const int64_t w0 = (debug & 32) ? pj_ns() : 0;
        while (pj.stA[tb].load(std::memory_order_acquire) < pj.nach)
          if (!pj_take_a()) HostPool::spin_pause();
        if (debug & 32) pj.ns_wait_a += pj_ns() - w0;
      }
      if (pj.offs) pj.offs[tb] = sa.used;
      pj.berr = pj_phaseB(tb);
      if (pj.berr) break;
      if (debug & 32) pj.b_clusters_extra += (sa.used - u0) != 3 * (int64_t)d;
      pj.stB[tb].store(1, std::memory_order_release);
    }
    if (pj.offs && !pj.berr) pj.offs[pj.T] = sa.used;
    pj.b_draws = sa.used - used0;
    pj.b_end = tb;
    pj.ns_b1.store(pj_ns());
    for (int t = tb; t < pj.T; ++t) pj.stB[t].store(-1, std::memory_order_release);
    return true;
  }
  void pj_work() {
    for (;;) {
      if (pj_fill()) continue;                    // the stream slice first: B waits on it
      if (pj_logit(PhiJob::kNSmall)) continue;    // the small first chunks: B's first draws
      if (pj_take_a(pj.t0 + 2)) continue;         // phase A of the first clusters
      if (pj_try_b()) continue;
      if (pj_logit()) continue;
      if (pj_take_a()) continue;
      if (pj.bclaim.load(std::memory_order_acquire) != 0) break;
      HostPool::spin_pause();                   // stream fill / logits in progress elsewhere
    }
    for (;;) {
      const int t = pj.nextC.fetch_add(1);
      if (t >= pj.T) break;
      int b;
      while ((b = pj.stB[t].load(std::memory_order_acquire)) == 0) HostPool::spin_pause();
      if (b < 0) break;                           // B stopped on an error
      if (!pj_phaseC(t)) {
        int cur = pj.gsl.load();
        while ((cur < 0 || t < cur) && !pj.gsl.compare_exchange_weak(cur, t)) {}
      }
    }
  }
  // Runs the prepared job on the pool and the calling thread; returns B's status.
  bool pj_open = false;
  void pj_launch() {
    HostPool& pool = HostPool::get();
    pj.t_launch = std::chrono::steady_clock::now();
    pj_open = pool.workers() > 0 && pool.try_launch([this](int) { pj_work(); });
  }
  int pj_finish() {
    pj_work();
    if (pj_open) HostPool::get().join();
    pj_open = false;
    return pj.berr;
  }

  // Started right after the sweep's draws are reserved, before its kernels are launched:
  // update_phi of every label on the pre-sweep state, into spec.*, on the pool while the
  // caller launches the sweep (spec_join collects it).  Its stream is phi_stream from the
  // sweep's end position; the chain's own Rng is not touched.
  void spec_launch() {
    spec.ran = false;
    spec.lv = 0;
    if (K <= 0) return;
    for (int k = 0; k < K; ++k)
      if (h_counts[k] <= 0) return;
    spec.K = K;
    spec.pos = rng.pos;
    spec.epoch = rng.epoch;
    spec.center = h_center;
    spec.sigma = h_sigma;
    spec.counts = h_counts;
    spec.off.assign((size_t)K + 1, 0);
    std::vector<int> touched(K);
    for (int k = 0; k < K; ++k) touched[k] = k;
    const UploadLayout L = stage_begin(K);
    stage_hold = spec.stage_buf = stage_fill;
    pj_setup(std::move(touched), 0, spec.counts.data(), h_freq.p, spec.center.data(), spec.sigma.data(), L, true,
             spec.off.data(), true);
    spec.moves = -1;
    spec.joined = false;
    pj_launch();
    spec.ran = true;
  }
  void spec_join() {
    if (!spec.ran) return;
    StreamAhead& sa = phi_stream;
    const int berr = pj_finish();
    int nv = berr ? pj.b_end : spec.K;
    const int gsl_t = pj.gsl.load();
    if (gsl_t >= 0) nv = std::min(nv, gsl_t);
    if (pj.failed || sa.n == 0 || sa.start.pos != spec.pos) nv = 0;
    if (sa.spilled)
      for (int t = 0; t < nv; ++t)
        if (spec.off[t + 1] > sa.n) { nv = t; break; }
    spec.nvalid = nv;
    if (debug & 32) {
      tsum("spec.fill_start", pj.ns_f0.load() * 1e-3);
      tsum("spec.state_at", pj.ns_f1.load() * 1e-3);
      tsum("spec.slice_at", pj.ns_f2.load() * 1e-3);
      tsum("spec.fill_at", pj.ns_fill.load() * 1e-3);
      tsum("spec.logits_at", pj.ns_logits.load() * 1e-3);
      tsum("spec.B_from", pj.ns_b0.load() * 1e-3);
      tsum("spec.B_to", pj.ns_b1.load() * 1e-3);
      tsum("spec.B_waitA", pj.ns_wait_a * 1e-3);
      tsum("spec.B_extra_draws", (double)(pj.b_draws - 3 * (int64_t)(pj.T - pj.t0) * d));
      tsum("spec.B_clusters_extra", (double)pj.b_clusters_extra);
      tsum("spec.B_waitL", pj.ns_wait_l * 1e-3);
      tsum("spec.joined_at", pj_ns() * 1e-3);
      tsum("spec.B_on_caller", pj.b_thread.load());
      std::snprintf(spec_line, sizeof(spec_line), " | spec fill %.0f state %.0f slice %.0f logits %.0f B %.0f-%.0f joined %.0f",
                    pj.ns_f0.load() * 1e-3, pj.ns_f1.load() * 1e-3, pj.ns_fill.load() * 1e-3,
                    pj.ns_logits.load() * 1e-3, pj.ns_b0.load() * 1e-3, pj.ns_b1.load() * 1e-3, pj_ns() * 1e-3);
    }
    // rewind: update_phi continues from spec.off[t0] of the same prefetched stream
    sa.used = 0;
    sa.spilled = false;
    sa.live = &rng;
    spec.moves = -1;
    spec.joined = true;
    stats.phi_spec_runs++;
  }

  // ------------------------------------------------------------------ update_phi on the device
  // csrc/phi.hip.  Static per-data arrays (m_j, their prefix sums, v, w, glibc tables), the
  // cluster descriptors and current sigmas of the update, scratch, and the outputs copied
  // back (status, centers, sigmas, log-likelihood terms).
  struct PhiDevice {
    bool ready = false;
    int sumatt = 0;
    DevBuf<int32_t> att, aoff;
    DevBuf<double> v, w;
    DevBuf<uint64_t> gtab;
    DevBuf<int> lab_cnt;               // [T] labels then [T] counts
    DevBuf<double> sig_in, sig_out, ll, cum;
    DevBuf<uint8_t> perm, det, pick, stage;
    DevBuf<PhiCand> cand;
    DevBuf<int> act, status;
    DevBuf<uint64_t> mask, maskd;
    DevBuf<uint8_t> ikind;
    DevBuf<int64_t> apos, dts;
    DevBuf<double> lg, lzz;
    DevBuf<int> F;
    DevBuf<uint16_t> tree;             // composition trees (tree mode)
    DevBuf<int> tnd;                   // per cluster: a pick depends on the uniform
    // fast path (launch_phi2): group and cluster tables, last-workgroup counters, the status
    // generation, and the inputs / outputs in coherent host memory (the kernels read and write
    // them directly: no copy commands on the update's path)
    DevBuf<uint16_t> gtab2, roots;
    DevBuf<int> ctr;
    DevBuf<unsigned long long> tdbg;
    int gen = 0;
    PinBuf<uint8_t> h_in2;
    DevBuf<uint8_t> d_in2;
    // by slot (consecutive fast updates alternate, so a chained update reads its predecessor's
    // labels, counts and sigmas on the device and writes its own tables and outputs beside
    // them): outputs + status + stream state in coherent host memory, staged tables, labels and
    // counts, sigmas, chain words
    PinBuf<uint8_t> out2[2];
    DevBuf<uint8_t> stage2[2];
    DevBuf<int> labc2[2];
    DevBuf<double> sigd2[2];
    DevBuf<PhiChain> chain2;
    int slot = 0;                      // the slot of the next fast update
    // the scratch (masks, tables, status) is shared by every update: one enqueued on another
    // stream than the last one waits for it (ev_last, recorded after each update's launch)
    hipEvent_t ev_last = nullptr;
    hipStream_t last_s = nullptr;
    bool fast_out(const uint8_t* o) const { return o && (o == out2[0].p || o == out2[1].p); }
    int64_t fast_calls = 0;
    // tree mode when every updated cluster has at least this many members (a small cluster's
    // center picks can depend on the uniform); raised past a cluster size that needed a retry
    int tree_min_count = 16;
    // fast path: a hand-back because a pick depended on the uniform (an unsettled chain) skips
    // the fast path for the next fast_backoff updates, then it is tried again
    int fast_backoff = 0;
    static constexpr int kFastBackoff = 16;
    PinBuf<uint8_t> h_in, h_out;
    double p_rej = 0.12;               // rbeta attempts rejected (window model), adapted per call
    double p_rej_sm = 0.12;            // the same for split-merge's one- or two-cluster updates
    // the estimate after an update with `drift` extra uniforms over `items` draws; a window
    // the drift left (kPhiShort / kPhiWindow) widens the next one
    // (the chain's estimate stays in [0.05, 0.3] as before: a wider window no longer fits the
    // LDS of wide rows' updates; split-merge's goes up to 0.9)
    static void adapt(double& p, int64_t drift, int64_t items, double hi = 0.3) {
      const double ph = (double)drift / ((double)drift + 2.0 * (double)items);
      p = std::min(hi, std::max(hi > 0.3 ? 0.02 : 0.05, 0.7 * p + 0.3 * ph));
    }
    static void widen(double& p, double hi = 0.3) { p = std::min(hi, 1.5 * p + 0.05); }
    int64_t calls = 0, fallbacks = 0;
    int last_status = 0;
  } phd;
  // update_phi placement: the host job speculated during the sweep (default), or the device
  // (phi.hip, after the sweep): HDPM_OPT_PHI_DEVICE, or HDPM_PHI=device in the environment;
  // debug bit 19 (value 524288) forces the host.
  // phi_mode: 0 the host job, 1 the device (fast path first), 2 the device's general kernels
  // only, 3 automatic (default): the device for the chain's update_phi when it has at least
  // kPhiAutoItems (cluster, attribute) items -- where the host job's serial draws outlast the
  // sweep (C4: 7,840 items, device 4.5k vs host 3.3k it/s) -- and the host job below that and for
  // split-merge's one- and two-cluster updates (C5 / C3: host 7.7k / 12.8k vs device 5.2k / 8.3k,
  // profiles/r06/ab_phi_auto/).  HDPM_PHI=host|device|device-general|auto overrides the default.
  static constexpr int64_t kPhiAutoItems = 4096;
  int phi_mode = [] {
    const char* e = std::getenv("HDPM_PHI");
    if (e && std::strcmp(e, "host") == 0) return 0;
    if (e && std::strcmp(e, "device") == 0) return 1;
    if (e && std::strcmp(e, "device-general") == 0) return 2;
    return 3;
  }();
  // update_phi of `items` (cluster, attribute) pairs of the chain on the device?
  bool phi_dev_for(int64_t items) const { return phi_mode == 1 || phi_mode == 2 || (phi_mode == 3 && items >= kPhiAutoItems); }
  bool host_spec() const { return !phi_dev_for((int64_t)K * d) || (debug & 524288); }
  double dev_ll = 0.0;                 // compute_loglikelihood from the last full device update
  uint64_t dev_ll_version = 0;         // labels_version it belongs to (0: none)

  void phi_device_setup() {
    if (phd.ready) return;
    std::vector<int32_t> off(d + 1, 0);
    for (int j = 0; j < d; ++j) off[j + 1] = off[j] + att[j];
    phd.sumatt = off[d];
    phd.att.ensure(d);
    phd.aoff.ensure(d + 1);
    phd.v.ensure(d);
    phd.w.ensure(d);
    phd.gtab.ensure(512);
    HIPCHK(hipMemcpy(phd.att.p, att.data(), (size_t)d * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(phd.aoff.p, off.data(), (size_t)(d + 1) * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(phd.v.p, v.data(), (size_t)d * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(phd.w.p, w.data(), (size_t)d * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(phd.gtab.p, glibc::kGlibcExpTab, 256 * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(phd.gtab.p + 256, glibc::kGlibcLogTab, 256 * 8, hipMemcpyHostToDevice));
    phd.ready = true;
  }

  // The window holding [pos, pos + n) and able to hand the host its state after it.
  RngWindow* window_at(uint64_t pos, int64_t n) {
    RngWindow* W = nullptr;
    for (auto& w_ : win)
      if (covers(w_, pos, n) && (!W || w_.start_pos < W->start_pos)) W = &w_;
    return W;
  }
  bool can_adopt(const RngWindow& W, uint64_t target) const {
    const uint64_t r = target - W.start_pos;
    const uint64_t head = W.mti0 >= 624 ? 0 : 624 - W.mti0;
    if (r < head) return true;
    const uint64_t b = 1 + (r - head) / 624, k = (r - head) % 624;
    const int64_t blk = (int64_t)(k == 0 ? b - 1 : b);
    return blk == 0 || blk >= W.export_from;
  }

  // update_phi (cf:511-591) of the labels in mask on the device.  Returns kOk when committed
  // (new centers / sigmas in h_center / h_sigma and in the device tables, the host stream
  // past the update's draws), -1 when the device path does not apply or met a case it
  // leaves to the host (nothing changed: same stream position, same tables).
  // Sizes of a device update of T clusters (phi.hip): drift windows (kernels.hpp phi_lo /
  // phi_hi, from the rate and spread of the extra uniforms per sigma draw), mask words per
  // candidate, start drifts walked per cluster, stream words read, walk workgroup shape.
  struct PhiPlan {
    bool ok = false;
    int T = 0, nw = 0, Wc = 0, wpb = 0, groups = 0, L = 0, S = 1;
    int64_t items = 0, need = 0;
    double rate = 0, sdev = 0;
    // composition trees (phi.hip k_phi_tree): tables of tW drifts, tnb level-0 blocks per
    // cluster, tSB blocks per workgroup, tS workgroups per cluster, tpc tables per cluster
    bool tree_ok = false;
    int tW = 0, tnb = 0, tSB = 0, tS = 0, tpc = 0, root_lds = 0;
    // fast path (launch_phi2): groups of gs items, G per cluster
    bool fast_ok = false;
    int gs = 0, G = 0;
  };
  // sd_scale < 1 narrows the drift windows (the fast path: kPhiFastSd standard deviations
  // instead of kPhiSd; a drift outside them is a window status and the update goes to the host)
  PhiPlan phi_plan(int T, bool sm = false, double sd_scale = 1.0) const {
    PhiPlan pl;
    if (T <= 0 || d > 2048) return pl;
    pl.T = T;
    const double p = sm ? phd.p_rej_sm : phd.p_rej;
    pl.rate = 2 * p / (1 - p);
    pl.sdev = sd_scale * 2 * std::sqrt(p) / (1 - p);
    pl.items = (int64_t)T * d;
    const int64_t klast = pl.items - 1;
    pl.nw = (int)((phi_hi(klast, pl.rate, pl.sdev) - phi_lo(klast, pl.rate, pl.sdev) + 63) / 64) + 3;
    pl.Wc = (int)(phi_hi(klast, pl.rate, pl.sdev) - phi_lo(klast, pl.rate, pl.sdev)) + 2;   // any segment start
    pl.need = 3 * pl.items + phi_hi(pl.items, pl.rate, pl.sdev) + 256;
    // LDS of the walks: the cluster image (d nw mask words) with the per-wave pick rows;
    // 16 waves per workgroup while that fits, fewer otherwise
    int wpb = 16;
    while (wpb > 1 && (phi_cwalk_lds(d, pl.nw, wpb) > 150 * 1024 || phi_values_lds(d, pl.nw) > 150 * 1024)) wpb /= 2;
    if (phi_cwalk_lds(d, pl.nw, wpb) > 150 * 1024 || phi_values_lds(d, pl.nw) > 150 * 1024) return pl;
    pl.wpb = wpb;
    // k_phi_cwalk: walk segments of at most 128 draws; kPhiIlp start drifts per thread, at
    // most 1024 threads per workgroup
    if (phi_cwalk_lds(d, pl.nw, 16) > 150 * 1024) return pl;
    pl.S = (d + 127) / 128;
    pl.L = (d + pl.S - 1) / pl.S;
    pl.groups = (pl.Wc + 1024 * phi_ilp() - 1) / (1024 * phi_ilp());
    pl.ok = true;
    // tree mode: the largest segment (<= 32 blocks of 4 items) whose tables fit the LDS
    pl.tW = 64 * (pl.nw - 1);
    pl.tnb = (d + 3) / 4;
    pl.tSB = 32;
    while (pl.tSB > 1 && phi_tree_lds_bytes(pl.tSB, pl.nw, pl.tW) > 150 * 1024) pl.tSB /= 2;
    pl.tS = (pl.tnb + pl.tSB - 1) / pl.tSB;
    pl.tpc = phi_loff(pl.tnb, phi_ltop(pl.tnb) + 1);
    pl.root_lds = phi_values2_lds_bytes(d, pl.tnb, T, pl.tW, pl.nw) <= 150 * 1024 ? 1 : 0;
    pl.tree_ok = pl.tW >= 64 && phi_tree_lds_bytes(pl.tSB, pl.nw, pl.tW) <= 150 * 1024 && pl.root_lds &&
                 pl.tW < 65535;
    // fast path: groups of gs items, k_phi2_group a workgroup per group.  The largest gs that
    // still gives >= 160 workgroups (their prep and masks run beside each other: more, smaller
    // groups contend for the CUs; fewer leave them idle), else the smallest that fits the LDS
    // (measured, one box, profiles/r06/phi2gs/: C4 T = 10, D = 784 -- gs 8 / 16 / 32 / 64: 6,512 /
    // 6,518 / 6,792 / 5,301 it/s; C5 with the device update, T = 20, D = 128 -- 8 / 16 / 32: 7,244 /
    // 7,566 / 7,163; C3, D = 64 -- 11,308 / 11,164 / 10,044).  HDPM_PHI2_GS forces one (testing).
    static const int gs_force = [] {
      const char* e = std::getenv("HDPM_PHI2_GS");
      const int v = e ? std::atoi(e) : 0;
      return (v == 8 || v == 16 || v == 32 || v == 64) ? v : 0;
    }();
    if (pl.tW >= 64 && pl.tW < 65535) {
      auto fits = [&](int gs) {
        const int G = (d + gs - 1) / gs;
        return phi2_tree_lds_bytes(T, G, pl.tW) <= 150 * 1024 && phi2_values_lds_bytes(d, G, pl.tW, T) <= 150 * 1024 &&
               phi2_group_lds_bytes(gs, pl.nw, pl.rate) <= 150 * 1024;
      };
      int pick = 0;
      if (gs_force) {
        if (fits(gs_force)) pick = gs_force;
      } else {
        for (int gs = 64; gs >= 8 && !pick; gs /= 2)
          if (fits(gs) && (int64_t)T * ((d + gs - 1) / gs) >= 160) pick = gs;
        for (int gs = 8; gs <= 64 && !pick; gs *= 2)
          if (fits(gs)) pick = gs;
      }
      if (pick) {
        pl.fast_ok = true;
        pl.gs = pick;
        pl.G = (d + pick - 1) / pick;
      }
    }
    return pl;
  }
  // scratch of a plan, and the arguments every call shares (the caller sets raw, labels /
  // counts, freq, sigmas in and out, outputs)
  PhiArgs phi_args(const PhiPlan& pl) {
    phi_device_setup();
    const int T = pl.T;
    const int64_t items = pl.items, cap = (int64_t)T * phd.sumatt;
    phd.cum.ensure((size_t)T * phd.sumatt);
    phd.perm.ensure((size_t)T * phd.sumatt);
    phd.cand.ensure((size_t)T * phd.sumatt);
    phd.det.ensure(items);
    phd.apos.ensure(items);
    phd.act.ensure(1 + 2 * cap);
    phd.mask.ensure((size_t)cap * pl.nw);
    phd.maskd.ensure((size_t)items * pl.nw);
    phd.ikind.ensure(items);
    phd.lg.ensure(pl.need);
    phd.lzz.ensure(pl.need);
    phd.F.ensure((size_t)T * pl.S * pl.Wc);
    phd.dts.ensure(T);
    PhiArgs a{};
    a.T = T; a.d = d; a.dp = dp; a.mmax = mmax; a.sumatt = phd.sumatt; a.wb = wb; a.Ws = Ws; a.bw = bw;
    a.att = phd.att.p; a.aoff = phd.aoff.p; a.v = phd.v.p; a.w = phd.w.p; a.gtab = phd.gtab.p;
    a.cum = phd.cum.p; a.perm = phd.perm.p; a.det = phd.det.p; a.cand = phd.cand.p;
    a.act = phd.act.p; a.nact_cap = cap; a.mask = phd.mask.p; a.nw = pl.nw; a.rate = pl.rate; a.sdev = pl.sdev;
    a.apos = phd.apos.p;
    a.lg = phd.lg.p; a.lzz = phd.lzz.p; a.span = pl.need - 1; a.F = phd.F.p; a.Wc = pl.Wc; a.dts = phd.dts.p;
    a.maskd = phd.maskd.p; a.ikind = phd.ikind.p; a.wpb = pl.wpb; a.groups = pl.groups; a.L = pl.L; a.S = pl.S;
    a.raw_ptr = nullptr; a.gate = nullptr; a.pos_in = nullptr; a.pos_out = nullptr; a.sweep_len = 0;
    a.slot_of = nullptr;
    a.tree = nullptr;
    a.tW = pl.tW; a.tnb = pl.tnb; a.tSB = pl.tSB; a.tS = pl.tS; a.tpc = pl.tpc; a.tRootLds = pl.root_lds;
    if (pl.tree_ok) {
      phd.tree.ensure((size_t)T * pl.tpc * pl.tW);
      phd.tnd.ensure(T);
    }
    a.tnd = phd.tnd.p;
    a.gs = 0; a.G = 0; a.gtab2 = nullptr; a.roots = nullptr; a.ctr = nullptr; a.gen = 0; a.status_host = nullptr;
    a.tdbg = nullptr;
    a.lab_dev = nullptr;
    return a;
  }

  // phi_mode 1: the fast path first where the plan allows it; 2: the general kernels only
  bool phi_fast(const PhiPlan& pl) const { return pl.fast_ok && phi_mode != 2; }
  // the fast path's plan (narrower windows), and whether it is taken for an update whose
  // smallest cluster has min_count members
  static constexpr double kPhiFastSd = 4.75;
  PhiPlan fast_plan(int T, bool sm, int min_count, bool* fast) {
    const PhiPlan pf = phi_plan(T, sm, kPhiFastSd / kPhiSd);
    *fast = phi_fast(pf) && min_count >= 16 && !(debug & 134217728);
    if (*fast && phd.fast_backoff > 0) {
      --phd.fast_backoff;
      *fast = false;
    }
    return pf;
  }

  // Enqueue one device update of T clusters on stream s: labels / counts / current sigmas in,
  // status + consumption, picks, sigmas and log-likelihood pairs out (phi_out_layout) in the
  // returned host buffer, complete once s reaches this point.  mode 2: the fast path
  // (launch_phi2: inputs and outputs in coherent host memory, no copy or fill commands);
  // 1: the general kernels with composition trees; 0: with the per-start-drift walks (both
  // with copies and fills around launch_phi).
  // chainW (mode 2 only): a chained update (PhiArgs::chain_in) behind the previous fast update
  // on s, its slice in window chainW after the previous update's end and sweep_len draws; lab,
  // cnt and sig_in are then unused (the previous update's, on the device).
  const uint8_t* enqueue_phi(PhiArgs& a, const PhiPlan& pl, int mode, const int* lab, const int* cnt,
                             const double* sig_in, hipStream_t s, hipEvent_t w1 = nullptr, hipEvent_t w2 = nullptr,
                             const RngWindow* chainW = nullptr, int64_t sweep_len = 0) {
    const int T = pl.T;
    const int64_t items = pl.items;
    size_t o_pick, o_sig, o_ll, bytes;
    phi_out_layout(T, d, &o_pick, &o_sig, &o_ll, &bytes);
    if (phd.last_s && phd.last_s != s) HIPCHK(hipStreamWaitEvent(s, phd.ev_last, 0));
    if (!phd.ev_last) HIPCHK(hipEventCreateWithFlags(&phd.ev_last, hipEventDisableTiming));
    phd.last_s = s;
    if (!phd.status.p) {
      // (zeroed in stream order: the fast path's generation-tagged words are never cleared, and
      // a hipMemset on the null stream is not ordered with these non-blocking streams)
      phd.status.ensure(4);
      HIPCHK(hipMemsetAsync(phd.status.p, 0, 16, s));
    }
    phd.stage.ensure(upload_layout(T, dp, d, bw).bytes);
    a.status = phd.status.p;
    a.stage = phd.stage.p;
    const size_t o_sigin = align16((size_t)2 * T * 4), in_bytes = o_sigin + (size_t)items * 8;
    if (mode == 2) {
      const size_t o_state = align16(bytes);             // the stream state after the update
      const int sl = phd.slot;
      phd.slot ^= 1;
      PinBuf<uint8_t>& hout = phd.out2[sl];
      hout.ensure(o_state + 625 * 4 + 64, hipHostMallocCoherent);
      phd.stage2[sl].ensure(upload_layout(T, dp, d, bw).bytes);
      a.stage = phd.stage2[sl].p;
      phd.labc2[sl].ensure(2 * T);
      phd.sigd2[sl].ensure(items);
      if (!phd.chain2.p) {
        phd.chain2.ensure(2);
        HIPCHK(hipMemsetAsync(phd.chain2.p, 0, 2 * sizeof(PhiChain), s));
      }
      a.chain_out = phd.chain2.p + sl;
      a.sig_dev = phd.sigd2[sl].p;
      a.lab_dev = phd.labc2[sl].p;   // (k_phi2_group's copy of the labels and counts for k_phi2_values)
      if (!phd.ctr.p) {
        phd.ctr.ensure(2);
        HIPCHK(hipMemsetAsync(phd.ctr.p, 0, 2 * sizeof(int), s));
      }
      phd.gtab2.ensure((size_t)T * pl.G * pl.tW);
      phd.roots.ensure((size_t)T * pl.tW);
      if (++phd.gen >= (1 << 26)) {                      // generations only grow: restart from 1
        HIPCHK(hipStreamSynchronize(s));
        HIPCHK(hipMemsetAsync(phd.status.p, 0, 16, s));
        phd.gen = 1;
      }
      ((volatile int*)hout.p)[0] = -1;                 // (written by the last k_phi2_values workgroup)
      if (chainW) {
        // the previous fast update's labels, counts and sigmas, its end position (device words)
        const int pv = sl ^ 1;
        a.lab = phd.labc2[pv].p; a.cnt = phd.labc2[pv].p + T; a.sig_in = phd.sigd2[pv].p;
        a.chain_in = phd.chain2.p + pv;
        a.win_raw = chainW->raw.p; a.win_start = (int64_t)chainW->start_pos; a.win_count = chainW->count;
        a.win_mti0 = chainW->mti0;
        a.sweep_len = sweep_len;
        a.raw = nullptr; a.nraw = 0; a.raw_back = 0; a.mti_pos = 0; a.pos0 = 0;
        if (w1) HIPCHK(hipStreamWaitEvent(s, w1, 0));
      } else {
        phd.h_in2.ensure(in_bytes + 64, hipHostMallocCoherent);
        int* hl = (int*)phd.h_in2.p;
        std::memcpy(hl, lab, (size_t)T * 4);
        std::memcpy(hl + T, cnt, (size_t)T * 4);
        std::memcpy(phd.h_in2.p + o_sigin, sig_in, (size_t)items * 8);
        // the inputs to the device in one copy, queued before the update's waits (the sweep's
        // scatter, the stream window) so it overlaps them: the kernels then read device memory
        // (a kernel's reads of host memory cost it a PCIe round trip each)
        phd.d_in2.ensure(in_bytes + 64);
        HIPCHK(hipMemcpyAsync(phd.d_in2.p, phd.h_in2.p, in_bytes, hipMemcpyHostToDevice, s));
        if (w1) HIPCHK(hipStreamWaitEvent(s, w1, 0));
        const int* dl = (const int*)phd.d_in2.p;
        a.lab = dl; a.cnt = dl + T; a.sig_in = (const double*)(phd.d_in2.p + o_sigin);
        a.chain_in = nullptr;
      }
      // (w2, the release of phd's buffers by the sweep's stream, guards the staging buffer:
      // only k_phi2_values writes it, so only it waits)
      a.pick = hout.p + o_pick;
      a.sig_out = (double*)(hout.p + o_sig);
      a.ll = (double*)(hout.p + o_ll);
      a.status_host = (int*)hout.p;
      a.state_host = a.raw_ptr == nullptr && (chainW || a.mti_pos >= 1) ? (uint32_t*)(hout.p + o_state) : nullptr;
      if (a.state_host) a.state_host[624] = 0;
      a.gs = pl.gs; a.G = pl.G; a.gtab2 = phd.gtab2.p; a.roots = phd.roots.p; a.ctr = phd.ctr.p; a.gen = phd.gen;
      a.tree = nullptr;
      a.lg = nullptr; a.lzz = nullptr;                   // the fast path computes its logits itself
      if (std::getenv("HDPM_PHI_TIMING")) {
        // testing: phase marks of the fast path (printed after a synchronous device update)
        if (!phd.tdbg.p) phd.tdbg.ensure(24);
        HIPCHK(hipMemsetAsync(phd.tdbg.p, 0, 24 * 8, s));
        a.tdbg = phd.tdbg.p;
      }
      HIPCHK(launch_phi2(a, s, w2));
      HIPCHK(hipEventRecord(phd.ev_last, s));
      phd.fast_calls++;
      stats.phi_fast_calls++;
      return hout.p;
    }
    if (w1) HIPCHK(hipStreamWaitEvent(s, w1, 0));
    if (w2) HIPCHK(hipStreamWaitEvent(s, w2, 0));
    a.stage = phd.stage.p;
    a.chain_in = nullptr; a.chain_out = nullptr; a.sig_dev = nullptr;
    phd.h_in.ensure(in_bytes + 64);
    phd.h_out.ensure(bytes);
    int* hl = (int*)phd.h_in.p;
    std::memcpy(hl, lab, (size_t)T * 4);
    std::memcpy(hl + T, cnt, (size_t)T * 4);
    std::memcpy(phd.h_in.p + o_sigin, sig_in, (size_t)items * 8);
    phd.lab_cnt.ensure(2 * T);
    phd.sig_in.ensure(items);
    phd.sig_out.ensure(items);
    phd.ll.ensure(2 * T);
    phd.pick.ensure(items);
    HIPCHK(hipMemcpyAsync(phd.lab_cnt.p, hl, (size_t)2 * T * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(phd.sig_in.p, phd.h_in.p + o_sigin, (size_t)items * 8, hipMemcpyHostToDevice, s));
    a.lab = phd.lab_cnt.p; a.cnt = phd.lab_cnt.p + T; a.sig_in = phd.sig_in.p;
    a.pick = phd.pick.p; a.sig_out = phd.sig_out.p; a.ll = phd.ll.p;
    a.status_host = nullptr;
    a.gen = 0;
    a.lg = phd.lg.p; a.lzz = phd.lzz.p;
    a.tree = mode == 1 ? phd.tree.p : nullptr;
    if (mode == 1) HIPCHK(hipMemsetAsync(phd.tnd.p, 0, (size_t)T * 4, s));
    HIPCHK(hipMemsetAsync(phd.status.p, 0, 16, s));
    HIPCHK(hipMemsetAsync(phd.act.p, 0, 4, s));
    HIPCHK(launch_phi(a, s));
    HIPCHK(hipMemcpyAsync(phd.h_out.p, phd.status.p, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(phd.h_out.p + o_pick, phd.pick.p, (size_t)items, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(phd.h_out.p + o_sig, phd.sig_out.p, (size_t)items * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(phd.h_out.p + o_ll, phd.ll.p, (size_t)2 * T * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipEventRecord(phd.ev_last, s));
    return phd.h_out.p;
  }

  int device_update_phi(const std::vector<unsigned char>& mask, int nidx) {
    if (phi_mode == 0 || (debug & (524288 | 64))) return -1;   // bit 19: host update_phi; bit 6: host pools
    if (phi_mode == 3) {                                  // automatic: by the update's size
      int64_t T0 = 0;
      for (int k = 0; k < K; ++k) T0 += mask[k] && h_counts[k] != 0;
      if (!phi_dev_for(T0 * d)) return -1;
    }
    if (!glibc_selfcheck() || d > 2048) return -1;
    std::vector<int> touched;
    for (int k = 0; k < K; ++k)
      if (mask[k] && h_counts[k] != 0) touched.push_back(k);
    const int T = (int)touched.size();
    if (T == 0) return -1;
    const bool full = tables_dirty || T == K;
    if (full && T != K) return -1;                        // untouched labels need the host's tables
    rng_sync();
    int min_count = INT_MAX;
    for (int t = 0; t < T; ++t) min_count = std::min(min_count, h_counts[touched[t]]);
    const PhiPlan pl = phi_plan(T);
    bool fast = false;
    const PhiPlan pf = fast_plan(T, false, min_count, &fast);
    if (!pl.ok) return -1;
    const int64_t items = pl.items, need = pl.need;
    dspec_drain();                                        // a speculation's use of phd is over
    RngWindow* W = window_at(rng.pos, need);
    if (!W) return -1;
    auto tp0 = std::chrono::steady_clock::now();
    histogram_launch(nidx == 0 ? nullptr : &mask);
    const unsigned* fsrc = nidx == 0 ? d_freq.p : d_freq_m.p;
    // inputs: labels, counts, current sigmas
    std::vector<int> labs(T), cnts(T);
    std::vector<double> sigs((size_t)items);
    for (int t = 0; t < T; ++t) {
      labs[t] = touched[t];
      cnts[t] = h_counts[touched[t]];
      std::memcpy(&sigs[(size_t)t * d], &h_sigma[(size_t)touched[t] * d], (size_t)d * 8);
    }
    size_t o_pick, o_sig, o_ll, obytes;
    phi_out_layout(T, d, &o_pick, &o_sig, &o_ll, &obytes);
    const uint8_t* out = nullptr;
    uint8_t* out_stage = nullptr;      // the staged tables of the update that produced `out`
    auto run = [&](int mode) {
      const PhiPlan& pm = mode == 2 ? pf : pl;
      PhiArgs a = phi_args(pm);
      a.freq = fsrc;
      phi_raw(a, *W);
      out = enqueue_phi(a, pm, mode, labs.data(), cnts.data(), sigs.data(), stream, W->done);
      out_stage = a.stage;
    };
    // the fast path, else the composition trees unless a cluster is small enough for a pick to
    // depend on the uniform (debug bit 27: always the per-start-drift walks)
    // (with one walk segment per cluster, d <= 128, such clusters are walked inside the tree-mode
    // update itself)
    const bool tree = pl.tree_ok && (pl.S == 1 || min_count >= phd.tree_min_count) && !(debug & 134217728);
    run(fast ? 2 : tree ? 1 : 0);
    histogram_wait(nidx == 0 ? nullptr : &mask);
    if (freq_next_pending) {
      std::swap(h_freq.p, h_freq_next.p);
      std::swap(h_freq.n, h_freq_next.n);
      freq_next_pending = false;
    }
    HIPCHK(hipStreamSynchronize(stream));
    phd.calls++;
    if (tree && !fast) stats.phi_tree_calls++;
    if (fast && phd.tdbg.p && std::getenv("HDPM_PHI_TIMING")) {
      unsigned long long m[24];
      HIPCHK(hipMemcpy(m, phd.tdbg.p, sizeof(m), hipMemcpyDeviceToHost));
      std::string line = "[phi2 us]";
      for (int q = 1; q < 23; ++q) {
        char b[32];
        std::snprintf(b, sizeof(b), " %d:%.2f", q, m[q] && m[0] ? (double)(long long)(m[q] - m[0]) * 0.01 : -1.0);
        line += b;
      }
      std::fprintf(stderr, "%s\n", line.c_str());
    }
    if (std::getenv("HDPM_PHI_TRACE"))
      std::fprintf(stderr, "[phi] T %d nw %d tW %d fast_ok %d gs %d G %d min_count %d tree_min %d fast %d tree %d status %d\n",
                   T, pl.nw, pl.tW, (int)pl.fast_ok, pl.gs, pl.G, min_count, phd.tree_min_count, (int)fast, (int)tree,
                   ((const int*)out)[0]);
    if (fast && ((const int*)out)[0] != kPhiOk) stats.phi_fast_handbacks++;
    if ((fast || tree) && ((const int*)out)[0] == kPhiNonDet) {
      // a pick depends on the uniform: the same update by the walks (same inputs, nothing
      // committed yet); updates with clusters this small take the walks directly from now on
      if (fast) phd.fast_backoff = PhiDevice::kFastBackoff;
      else phd.tree_min_count = std::max(phd.tree_min_count, std::min(1 << 20, 2 * min_count));
      stats.phi_tree_retries++;
      run(0);
      HIPCHK(hipStreamSynchronize(stream));
    } else if (fast && ((const int*)out)[0] != kPhiOk && ((const int*)out)[0] != kPhiWindow &&
               ((const int*)out)[0] != kPhiShort) {
      // a case the fast path leaves to the general kernels (the bisection path, ...)
      run(tree ? 1 : 0);
      HIPCHK(hipStreamSynchronize(stream));
    }
    const int status = ((const int*)out)[0];
    stats.phi_device_last_status = status;
    int64_t cons = 0;
    std::memcpy(&cons, out + 8, 8);
    phd.last_status = status;
    const uint64_t target = rng.pos + (uint64_t)cons;
    if ((debug & 2) && !fast) {
      std::vector<int64_t> dts(T);
      HIPCHK(hipMemcpy(dts.data(), phd.dts.p, (size_t)T * 8, hipMemcpyDeviceToHost));
      std::vector<int> F((size_t)T * pl.S * pl.Wc);
      HIPCHK(hipMemcpy(F.data(), phd.F.p, F.size() * 4, hipMemcpyDeviceToHost));
      int valid0 = 0;
      for (int c = 0; c < pl.Wc; ++c) valid0 += F[c] >= 0;
      std::string vs;
      for (int t = 0; t < T; ++t) {
        int v = 0, lo = -1, hi = -1;
        for (int c = 0; c < pl.Wc; ++c)
          if (F[(size_t)t * pl.S * pl.Wc + c] >= 0) { v++; if (lo < 0) lo = c; hi = c; }
        vs += " t" + std::to_string(t) + ":" + std::to_string(v) + "[" + std::to_string(lo) + "," + std::to_string(hi) +
              "] F0 " + std::to_string(F[(size_t)t * pl.S * pl.Wc]) + " Fmid " + std::to_string(F[(size_t)t * pl.S * pl.Wc + pl.Wc / 2]) +
              "] dts " + std::to_string(dts[t]) + " clo " + std::to_string(phi_lo((int64_t)t * d, pl.rate, pl.sdev));
      }
      std::fprintf(stderr, "[phi] F%s\n", vs.c_str());
      std::fprintf(stderr, "[phi] T %d nw %d Wc %d status %d cons %lld dts0 %lld F[0][0] %d valid(t=0) %d rate %.4f sdev %.4f\n",
                   T, pl.nw, pl.Wc, status, (long long)cons, (long long)dts[0], F[0], valid0, pl.rate, pl.sdev);
    }
    if (status != kPhiOk || cons <= 0 || !can_adopt(*W, target)) {
      phd_release(stream);
      phd.fallbacks++;
      stats.phi_device_fallbacks++;
      stats.phi_fallback_status_mask |= (int64_t)1 << (status != kPhiOk ? std::min(std::max(status, 0), 14) : 15);
      if (status == kPhiOk) stats.phi_device_last_status = -1;
      return -1;
    }
    stats.phi_device_calls++;
    // commit: tables on the device, parameters on the host, the stream past the draws
    HIPCHK(launch_scatter_clusters(out_stage, T, dp, d, bw, full ? 1 : 0, d_slot_codes.p, d_slot_tab.p, d_slot_bnd.p,
                                   d_counts.p, d_sol.p, d_los.p, d_src.p, stream));
    phd_release(stream);
    const uint8_t* pk = out + o_pick;
    const double* sg = (const double*)(out + o_sig);
    const double* ll = (const double*)(out + o_ll);
    double hi = 0.0, lo = 0.0;
    for (int t = 0; t < T; ++t) {
      const int k = touched[t];
      for (int j = 0; j < d; ++j) h_center[(size_t)k * d + j] = (uint8_t)(pk[(size_t)t * d + j] + 1);
      std::memcpy(&h_sigma[(size_t)k * d], sg + (size_t)t * d, (size_t)d * 8);
      for (int q = 0; q < 2; ++q) {
        const double x = ll[2 * t + q], s = hi + x;
        lo += std::fabs(hi) >= std::fabs(x) ? (hi - s) + x : (x - s) + hi;
        hi = s;
      }
    }
    if (full) {
      dev_ll = hi + lo;
      dev_ll_version = labels_version;
      tables_dirty = false;
    }
    stage_full = false;                // the host staging no longer mirrors the device tables
    adopt_after_phi(*W, target, phd.fast_out(out) ? (const uint32_t*)(out + phi_state_off(T, d)) : nullptr);
    // the drift model follows the chain: extra uniforms per sigma draw seen here
    PhiDevice::adapt(phd.p_rej, cons - 3 * items, items);
    stats.t_host_phi_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp0).count();
    return kOk;
  }

  // ------------------------------------------------------------------ update_phi speculated on the device
  // phi_mode 1: the update of the pre-sweep state (every label with its count, frequency
  // table and sigmas) is launched on pstream beside the sweep, at the stream position after the
  // sweep's draws (a sweep consumes exactly N (m + 1) uniforms) -- the device counterpart of
  // spec_launch.  A sweep that moves no point leaves all of its inputs as they were, so the
  // speculation is then update_phi itself (dspec_commit); after a sweep with moves it is dropped
  // and update_phi runs on the sweep's result.  phd's buffers are shared with device_update_phi:
  // every device use of them on the sweep's stream records ev_phd_free, which the next
  // speculation waits for, and device_update_phi waits for the speculation (dspec.ev).
  struct DevSpec {
    bool ran = false;                  // launched for the sweep whose draws end at pos
    bool inflight = false;             // launched and not yet waited for on the host
    uint64_t pos = 0, epoch = 0, lv = 0;
    int K = 0;
    int moves = -1;                    // the sweep's moves (set at its end)
    PhiPlan pl;
    RngWindow* W = nullptr;
    bool tree = false;
    size_t o_pick = 0, o_sig = 0, o_ll = 0;
    const uint8_t* out = nullptr;      // its outputs (phd.h_out, or phd.out2[slot] on the fast path)
    bool fast = false;
    hipEvent_t ev = nullptr;           // they are complete
    uint8_t* stage = nullptr;          // its staged tables
    int gen = 0;                       // fast path: its status generation
    int prev_gen = 0;                  // chained: the update it follows
    uint64_t est_pos = 0;              // chained: its nominal first position (when launched)
    uint64_t wgen = 0;                 // W's generation when launched
    int64_t sweep_len = 0;             // chained: the sweep's draws before it
    PhiChain* chain = nullptr;         // fast path: its chain word (end position, completion)
  } dspec, dnext;
  // dnext: the fast update after dspec's, enqueued behind it on pstream before dspec ran
  // (chained, PhiArgs::chain_in): the update of the iteration after next, valid when the sweep
  // between them moves nothing and dspec's update is the one committed (pipe_go promotes it)
  int committed_gen = 0;               // the fast update update_phi committed last (0: another)
  bool phi_chain = true;               // HDPM_PHI_CHAIN=0: no chained updates
  hipEvent_t ev_phd_free = nullptr;    // the last device use of phd's buffers on `stream` is done
  bool dspec_on() const { return phi_dev_for((int64_t)K * d) && !(debug & (524288 | 64 | 128)); }
  void phd_release(hipStream_t s) {
    if (!ev_phd_free) HIPCHK(hipEventCreateWithFlags(&ev_phd_free, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ev_phd_free, s));
  }
  void dspec_wait() {
    if (!dspec.inflight) return;
    if (dspec.fast) {
      // the fast path's last workgroup writes the status word last (system-scope release, after
      // every other output and after every other workgroup finished): spin on it instead of a
      // blocking event wait (whose wake-up alone costs tens of microseconds); 2 s, then the event
      const auto t0 = std::chrono::steady_clock::now();
      for (int polls = 0;; ++polls) {
        if (__atomic_load_n((const int*)dspec.out, __ATOMIC_ACQUIRE) != -1) break;
        HostPool::spin_pause();
        if ((polls & 1023) == 1023 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
          HIPCHK(hipEventSynchronize(dspec.ev));
          break;
        }
      }
    } else {
      HIPCHK(hipEventSynchronize(dspec.ev));
    }
    dspec.inflight = false;
  }
  // outputs of a device update of T clusters in phd.h_out: status + consumption, picks, sigmas,
  // log-likelihood pairs
  static void phi_out_layout(int T, int d_, size_t* o_pick, size_t* o_sig, size_t* o_ll, size_t* bytes) {
    const size_t items = (size_t)T * d_;
    *o_pick = 16;
    *o_sig = align16(*o_pick + items);
    *o_ll = *o_sig + items * 8;
    *bytes = *o_ll + (size_t)2 * T * 8;
  }
  // (the fast path's copy of the stream state follows them)
  static size_t phi_state_off(int T, int d_) {
    size_t o_pick, o_sig, o_ll, bytes;
    phi_out_layout(T, d_, &o_pick, &o_sig, &o_ll, &bytes);
    return align16(bytes);
  }

  void dspec_launch() {
    dspec.ran = false;
    if (!dspec_on() || K <= 0 || d > 2048 || !glibc_selfcheck()) return;
    int min_count = INT_MAX;
    for (int k = 0; k < K; ++k) {
      if (h_counts[k] <= 0) return;
      min_count = std::min(min_count, h_counts[k]);
    }
    bool fast = false;
    const PhiPlan pf = fast_plan(K, false, min_count, &fast);
    const PhiPlan pl = fast ? pf : phi_plan(K);
    if (std::getenv("HDPM_PHI_TRACE"))
      std::fprintf(stderr, "[phi dspec launch] T %d p_rej %.4f nw %d tW %d fast_ok %d gs %d G %d min_count %d tree_min %d fast %d\n",
                   K, phd.p_rej, pf.nw, pf.tW, (int)pf.fast_ok, pf.gs, pf.G, min_count, phd.tree_min_count, (int)fast);
    if (!pl.ok) return;
    RngWindow* W = window_at(rng.pos, pl.need);
    if (!W) return;
    dspec_wait();                      // phd.h_in / h_out are free on the host
    PhiArgs a = phi_args(pl);
    const int T = K;
    size_t bytes;
    phi_out_layout(T, d, &dspec.o_pick, &dspec.o_sig, &dspec.o_ll, &bytes);
    std::vector<int> labs(T);
    for (int t = 0; t < T; ++t) labs[t] = t;
    if (!dspec.ev) HIPCHK(hipEventCreateWithFlags(&dspec.ev, hipEventDisableTiming));

    a.freq = d_freq.p;
    phi_raw(a, *W);
    const bool tree = pl.tree_ok && (pl.S == 1 || min_count >= phd.tree_min_count) && !(debug & 134217728);
    dnext.ran = false;                 // (a chained update still queued completes unused)
    dspec.out = enqueue_phi(a, pl, fast ? 2 : tree ? 1 : 0, labs.data(), h_counts.data(), h_sigma.data(), pstream,
                            W->done, ev_phd_free);
    HIPCHK(hipEventRecord(dspec.ev, pstream));
    dspec.stage = a.stage;
    dspec.gen = fast ? a.gen : 0;
    dspec.prev_gen = 0;
    dspec.wgen = W->gen;
    dspec.chain = fast ? a.chain_out : nullptr;
    dspec.ran = true;
    dspec.inflight = true;
    dspec.pos = rng.pos;
    dspec.epoch = rng.epoch;
    dspec.lv = 0;
    dspec.K = K;
    dspec.moves = -1;
    dspec.pl = pl;
    dspec.W = W;
    dspec.tree = tree && !fast;
    dspec.fast = fast;
    stats.phi_dspec_launched++;
  }

  // Every speculation's use of phd's buffers is over (dspec and a chained dnext).
  void dspec_drain() {
    dspec_wait();
    if (dnext.inflight) {
      HIPCHK(hipEventSynchronize(dnext.ev));
      dnext.inflight = false;
    }
    dnext.ran = false;
  }

  // The chained update after dspec's (fast path): enqueued now, behind dspec on pstream, before
  // dspec ran.  Its first draw follows dspec's end and the next sweep's N (m + 1) draws (found on
  // the device: k_phi2_* read dspec's chain word), its inputs are dspec's outputs (labels,
  // counts, sigmas on the device), in the window that holds the nominal stretch; it runs only if
  // dspec completed.  pipe_go makes it the next iteration's speculation (dspec_promote).
  void dnext_launch(int m) {
    dnext.ran = false;
    static const bool env_off = [] {
      const char* e = std::getenv("HDPM_PHI_CHAIN");
      return e && e[0] == '0';
    }();
    if (!phi_chain || env_off || !dspec.ran || !dspec.fast || !dspec.inflight || dspec.gen != phd.gen ||
        phd.fast_backoff > 0 || K <= 0)
      return;
    const PhiPlan pl = phi_plan(K, false, kPhiFastSd / kPhiSd);
    if (!pl.ok || !phi_fast(pl)) return;
    const int64_t sweep_len = (int64_t)n * (m + 1);
    const uint64_t lo = dspec.pos + 3 * (uint64_t)dspec.pl.items + (uint64_t)sweep_len;   // >= 3 draws per item
    const uint64_t hi = dspec.pos + (uint64_t)dspec.pl.need + (uint64_t)sweep_len + (uint64_t)pl.need;
    RngWindow* W = window_at(lo, (int64_t)(hi - lo));
    if (!W) return;
    PhiArgs a = phi_args(pl);
    a.freq = d_freq.p;
    if (!dnext.ev) HIPCHK(hipEventCreateWithFlags(&dnext.ev, hipEventDisableTiming));
    dnext.out = enqueue_phi(a, pl, 2, nullptr, nullptr, nullptr, pstream, W->done, ev_phd_free, W, sweep_len);
    HIPCHK(hipEventRecord(dnext.ev, pstream));
    dnext.ran = true;
    dnext.inflight = true;
    dnext.pos = 0;                     // (known when dspec's update is committed)
    dnext.epoch = rng.epoch;
    dnext.lv = 0;
    dnext.K = K;
    dnext.moves = -1;
    dnext.pl = pl;
    dnext.W = W;
    dnext.wgen = W->gen;
    dnext.tree = false;
    dnext.fast = true;
    dnext.stage = a.stage;
    dnext.chain = a.chain_out;
    dnext.gen = a.gen;
    dnext.prev_gen = dspec.gen;
    dnext.est_pos = lo;
    dnext.sweep_len = sweep_len;
    dnext.o_pick = dspec.o_pick;
    dnext.o_sig = dspec.o_sig;
    dnext.o_ll = dspec.o_ll;
    stats.phi_chain_launched++;
  }
  // pipe_go (the sweep enqueued ahead goes, dspec's update committed): the chained update
  // becomes the speculation of the sweep now going when it follows the committed update
  bool dspec_promote(int m) {
    if (!dnext.ran) return false;
    dnext.ran = false;
    const bool ok = committed_gen != 0 && dnext.prev_gen == committed_gen && dnext.K == K &&
                    dnext.epoch == rng.epoch && dnext.sweep_len == (int64_t)n * (m + 1) && dnext.W &&
                    dnext.W->gen == dnext.wgen && covers(*dnext.W, rng.pos, dnext.pl.need) && dspec_on() &&
                    !dspec.inflight;
    if (!ok) {
      stats.phi_chain_dropped++;
      return false;
    }
    std::swap(dspec, dnext);
    dspec.ran = true;
    dspec.pos = rng.pos;
    dspec.lv = 0;
    dspec.moves = -1;
    dnext.ran = false;
    dnext.inflight = false;
    stats.phi_dspec_launched++;
    return true;
  }

  // The tables of the committed speculation, from phd.stage into the slots (full upload).
  void scatter_dev_stage(int T) {
    HIPCHK(hipStreamWaitEvent(stream, dspec.ev, 0));
    HIPCHK(launch_scatter_clusters(dspec.stage, T, dp, d, bw, 1, d_slot_codes.p, d_slot_tab.p, d_slot_bnd.p, d_counts.p,
                                   d_sol.p, d_los.p, d_src.p, stream));
    phd_release(stream);
  }

  // update_phi from the speculation (after a sweep without moves): kOk, or -1 when it did not
  // complete on the device (the caller runs the update; nothing was changed).
  int dspec_commit() {
    dspec_wait();
    dspec.ran = false;
    phd.calls++;
    if (dspec.tree) stats.phi_tree_calls++;
    const int T = dspec.K;
    const int status = ((const int*)dspec.out)[0];
    if (dspec.fast && status != kPhiOk) stats.phi_fast_handbacks++;
    if (std::getenv("HDPM_PHI_TRACE"))
      std::fprintf(stderr, "[phi dspec] T %d fast %d status %d\n", T, (int)dspec.fast, status);
    stats.phi_device_last_status = status;
    int64_t cons = 0;
    std::memcpy(&cons, dspec.out + 8, 8);
    const uint64_t target = rng.pos + (uint64_t)cons;
    if (status == kPhiNonDet) {
      if (dspec.fast) {
        phd.fast_backoff = PhiDevice::kFastBackoff;
      } else {
        int mc = INT_MAX;
        for (int k = 0; k < T; ++k) mc = std::min(mc, h_counts[k]);
        phd.tree_min_count = std::max(phd.tree_min_count, std::min(1 << 20, 2 * mc));
      }
    }
    // a sweep the device already started behind this update (PipeAuto) is followed: the update
    // completed with its stream state (the chain word), so the host takes it as it is
    const bool followed = pre_dev_decision() == 1;
    if (followed && (status != kPhiOk || cons <= 0 || !dspec.W)) {
      (void)hipStreamSynchronize(stream);
      have_state = false;
      err = "a sweep went ahead on the device behind an update the host cannot take";
      stats.pipe_desync++;
      return -1;
    }
    if (!followed && (status != kPhiOk || cons <= 0 || !dspec.W || dspec.W->gen != dspec.wgen ||
                      !can_adopt(*dspec.W, target) || !covers(*dspec.W, rng.pos, dspec.pl.need))) {
      phd.fallbacks++;
      stats.phi_device_fallbacks++;
      stats.phi_fallback_status_mask |= (int64_t)1 << (status != kPhiOk ? std::min(std::max(status, 0), 14) : 15);
      return -1;
    }
    stats.phi_device_calls++;
    stats.phi_dspec_used++;
    if (dspec.prev_gen) stats.phi_chain_used++;
    committed_gen = dspec.fast ? dspec.gen : 0;
    const uint32_t* st_words = dspec.fast ? (const uint32_t*)(dspec.out + phi_state_off(T, d)) : nullptr;
    // tables: by the sweep enqueued ahead (its gated scatter, pipe_go), flush_commit, or now
    if (defer_commit) {
      commit_later.active = true;
      commit_later.dev = true;
      commit_later.nent = T;
    } else {
      scatter_dev_stage(T);
    }
    const uint8_t* pk = dspec.out + dspec.o_pick;
    const double* sg = (const double*)(dspec.out + dspec.o_sig);
    const double* ll = (const double*)(dspec.out + dspec.o_ll);
    double hi = 0.0, lo = 0.0;
    for (int t = 0; t < T; ++t) {
      for (int j = 0; j < d; ++j) h_center[(size_t)t * d + j] = (uint8_t)(pk[(size_t)t * d + j] + 1);
      for (int q = 0; q < 2; ++q) {
        const double x = ll[2 * t + q], s2 = hi + x;
        lo += std::fabs(hi) >= std::fabs(x) ? (hi - s2) + x : (x - s2) + hi;
        hi = s2;
      }
    }
    std::memcpy(h_sigma.data(), sg, (size_t)T * d * 8);
    dev_ll = hi + lo;
    dev_ll_version = labels_version;
    tables_dirty = false;
    stage_full = false;                // the host staging no longer mirrors the device tables
    freq_next_pending = false;
    freq_version = labels_version;
    adopt_after_phi(*dspec.W, target, st_words);
    PhiDevice::adapt(phd.p_rej, cons - 3 * dspec.pl.items, dspec.pl.items);
    return kOk;
  }

  // update_phi (cf:511-591) of T clusters of a split-merge state on the device (sm:221, sm:387,
  // sm:584): their sizes `cnt`, frequency tables `freq` ([T][d][mmax], the move's host tables) and
  // current sigmas; the new centers (codes) and sigmas into cen / sig ([T][d]).  kOk, or -1
  // when the device path does not apply or hands the update back (nothing changed: same
  // stream position).  The host stream is synchronised to the position after the draws.
  DevBuf<unsigned> d_sm_freq;
  PinBuf<unsigned> h_sm_freq;
  int device_update_phi_sm(int T, const int* cnt, const unsigned* freq, const double* sig_in, uint8_t* cen,
                           double* sig) {
    // (automatic mode: split-merge's updates stay on the host job)
    if (phi_mode == 0 || phi_mode == 3 || (debug & (524288 | 64)) || T <= 0 || d > 2048 || !glibc_selfcheck()) return -1;
    rng_sync();
    // a drift past the window (a merged or freshly split cluster can reject far more attempts
    // than the chain's updates; nothing was consumed) is retried with a wider window
    for (int attempt = 0;; ++attempt) {
      const int r = device_update_phi_sm_once(T, cnt, freq, sig_in, cen, sig);
      if (r == 1 && attempt >= 2) {
        phd.fallbacks++;
        stats.phi_device_fallbacks++;
        return -1;
      }
      if (r != 1) return r;
      stats.phi_sm_window_retries++;
    }
  }
  // kOk, -1 (handed back), or 1: the drift left the window (widened for the next attempt)
  int device_update_phi_sm_once(int T, const int* cnt, const unsigned* freq, const double* sig_in, uint8_t* cen,
                                double* sig) {
    int min_count = INT_MAX;
    for (int t = 0; t < T; ++t) min_count = std::min(min_count, cnt[t]);
    const PhiPlan pl = phi_plan(T, true);
    bool fast = false;
    const PhiPlan pf = fast_plan(T, true, min_count, &fast);
    if (!pl.ok) return -1;
    RngWindow* W = window_at(rng.pos, pl.need);
    if (!W) return -1;
    dspec_drain();
    const int64_t items = pl.items;
    const size_t fw = (size_t)T * d * mmax;
    h_sm_freq.ensure(fw);
    d_sm_freq.ensure(fw);
    std::memcpy(h_sm_freq.p, freq, fw * 4);
    std::vector<int> labs(T);
    for (int t = 0; t < T; ++t) labs[t] = t;
    size_t o_pick, o_sig, o_ll, bytes;
    phi_out_layout(T, d, &o_pick, &o_sig, &o_ll, &bytes);
    HIPCHK(hipMemcpyAsync(d_sm_freq.p, h_sm_freq.p, fw * 4, hipMemcpyHostToDevice, stream));
    const uint8_t* out = nullptr;
    auto run = [&](int mode) {
      const PhiPlan& pm = mode == 2 ? pf : pl;
      PhiArgs a = phi_args(pm);
      a.freq = d_sm_freq.p;
      phi_raw(a, *W);
      out = enqueue_phi(a, pm, mode, labs.data(), cnt, sig_in, stream, W->done);
      HIPCHK(hipStreamSynchronize(stream));
    };
    const bool tree = pl.tree_ok && (pl.S == 1 || min_count >= phd.tree_min_count) && !(debug & 134217728);
    run(fast ? 2 : tree ? 1 : 0);
    phd.calls++;
    if (tree && !fast) stats.phi_tree_calls++;
    if (fast && ((const int*)out)[0] != kPhiOk) stats.phi_fast_handbacks++;
    if ((fast || tree) && ((const int*)out)[0] == kPhiNonDet) {
      if (fast) phd.fast_backoff = PhiDevice::kFastBackoff;
      else phd.tree_min_count = std::max(phd.tree_min_count, std::min(1 << 20, 2 * min_count));
      stats.phi_tree_retries++;
      run(0);
    } else if (fast && ((const int*)out)[0] != kPhiOk && ((const int*)out)[0] != kPhiWindow &&
               ((const int*)out)[0] != kPhiShort) {
      run(tree ? 1 : 0);
    }
    phd_release(stream);
    const int status = ((const int*)out)[0];
    stats.phi_device_last_status = status;
    int64_t cons = 0;
    std::memcpy(&cons, out + 8, 8);
    const uint64_t target = rng.pos + (uint64_t)cons;
    if (status != kPhiOk || cons <= 0 || !can_adopt(*W, target)) {
      stats.phi_fallback_status_mask |= (int64_t)1 << (status != kPhiOk ? std::min(std::max(status, 0), 14) : 15);
      if (status == kPhiOk) stats.phi_device_last_status = -1;
      if (status != kPhiShort && status != kPhiWindow) {
        phd.fallbacks++;
        stats.phi_device_fallbacks++;
      }
      if (std::getenv("HDPM_PHI_TRACE"))
        std::fprintf(stderr, "[phi sm] T %d items %lld need %lld nw %d p_rej %.4f status %d cons %lld counts %d %d\n", T,
                     (long long)items, (long long)pl.need, pl.nw, phd.p_rej_sm, status, (long long)cons, cnt[0],
                     T > 1 ? cnt[1] : -1);
      if (status == kPhiShort || status == kPhiWindow) {
        const double p0 = phd.p_rej_sm;
        PhiDevice::widen(phd.p_rej_sm, 0.9);
        if (phd.p_rej_sm > p0) return 1;   // a wider window is worth another try
        phd.fallbacks++;
        stats.phi_device_fallbacks++;
      }
      return -1;
    }
    stats.phi_device_calls++;
    stats.phi_sm_device_calls++;
    const uint8_t* pk = out + o_pick;
    for (int64_t q = 0; q < items; ++q) cen[q] = (uint8_t)(pk[q] + 1);
    std::memcpy(sig, out + o_sig, (size_t)items * 8);
    adopt_after_phi(*W, target, phd.fast_out(out) ? (const uint32_t*)(out + phi_state_off(T, d)) : nullptr);
    rng_sync();                        // split-merge draws on the host next
    PhiDevice::adapt(phd.p_rej_sm, cons - 3 * items, items, 0.9);
    return kOk;
  }

  int update_phi(const int32_t* idx, int nidx) {
    if (!have_state) { err = "no state"; return kArg; }
    // the log-likelihood a full device update summed belongs to the parameters before this
    // update: only a full device commit below sets it again (and the chained update follows
    // only a committed speculation)
    dev_ll_version = 0;
    committed_gen = 0;
    HostPool& pool = HostPool::get();
    pool.prewake();                                   // workers spin while the device counts
    auto t0c = std::chrono::steady_clock::now();
    std::vector<unsigned char> mask(K, nidx == 0 ? 1 : 0);
    for (int q = 0; q < nidx; ++q)
      if (idx[q] >= 0 && idx[q] < K) mask[idx[q]] = 1;
    StreamAhead& sa = phi_stream;
    // speculation of the sweep just done (spec_launch), for the full update only
    const bool use_spec = nidx == 0 && spec.ran && spec.lv == labels_version && spec.moves >= 0 &&
                          spec.pos == rng.pos && spec.epoch == rng.epoch && sa.n > 0 && sa.start.pos == rng.pos &&
                          !(debug & 128);
    spec.ran = false;
    // the device speculation of the sweep just done (dspec_launch)
    const bool use_dspec = nidx == 0 && dspec.ran && dspec.lv == labels_version && dspec.moves == 0 &&
                           dspec.pos == rng.pos && dspec.epoch == rng.epoch && K == dspec.K && dspec_on();
    if (pre.active && !(use_spec && spec.moves == 0 && K == spec.K && spec.nvalid == K) && !use_dspec) pre_release();
    if (use_dspec) {
      mark("dspec_wait");
      if (dspec_commit() == kOk) {
        stats.t_host_phi_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0c).count();
        mark("dspec");
        return kOk;
      }
      if (pre.active) pre_release();
    }
    dspec.ran = false;
    if (!use_spec) {
      // the update on the device (csrc/phi.hip); -1: not applicable here, the host runs it
      const int st = device_update_phi(mask, nidx);
      if (st >= 0) return st;
    }
    int t0 = 0;
    if (use_spec && spec.moves == 0 && K == spec.K) {
      // nothing moved: the frequency tables are the pre-sweep ones (the sweep's copy-out,
      // still in flight, has the same contents) -- no wait for the device
      t0 = spec.nvalid;
      freq_next_pending = false;
      freq_version = labels_version;
      rng_sync();
      mark("hist_wait");
    } else {
      histogram_launch(nidx == 0 ? nullptr : &mask);
      mark("hist_launch");
      // while the device counts: the next stretch of the stream and its logits (usually
      // already generated during the sweep)
      if (!use_spec) prefill_phi_stream();
      mark("prefill");
      histogram_wait(nidx == 0 ? nullptr : &mask);
      if (use_spec && freq_next_pending) {
        // the leading labels the sweep left alone: same slot and count (spec.pfx), same table
        const size_t row = (size_t)d * mmax;
        int pfx = std::min(spec.pfx, spec.nvalid);
        for (int l = 0; l < pfx; ++l)
          if (std::memcmp(h_freq.p + l * row, h_freq_next.p + l * row, row * 4) != 0) { pfx = l; break; }
        t0 = pfx;
      }
      if (freq_next_pending) {
        std::swap(h_freq.p, h_freq_next.p);
        std::swap(h_freq.n, h_freq_next.n);
        freq_next_pending = false;
      }
      mark("hist_wait");
    }
    if (use_spec) {
      sa.used = spec.off[t0];
      sa.spilled = false;
      sa.live = &rng;
      for (int k = 0; k < t0; ++k) {
        std::memcpy(&h_center[(size_t)k * d], &spec.center[(size_t)k * d], d);
        std::memcpy(&h_sigma[(size_t)k * d], &spec.sigma[(size_t)k * d], (size_t)d * 8);
      }
      stats.phi_spec_clusters += t0;
    } else {
      sa.live = &rng;
    }
    auto t1 = std::chrono::steady_clock::now();
    std::vector<int> touched;
    for (int i = 0; i < K; ++i)
      if (mask[i] && h_counts[i] != 0) touched.push_back(i);
    const int T = (int)touched.size();
    if (t0 > T) t0 = T;
    // staging of the new tables: all labels when every label is updated (or the device
    // tables are stale), else the touched ones
    const bool full = tables_dirty || T == K;
    if (full) ensure_slots(K + 2);
    const int nent = full ? K : T;
    // the speculation staged its clusters into spec.stage_buf (held since): same layout
    // when every label is staged and K did not change
    const bool spec_layout = use_spec && t0 > 0 && full && K == spec.K && spec.stage_buf == stage_hold;
    UploadLayout L;
    if (spec_layout) {
      L = upload_layout(K, dp, d, bw);
      stage_fill = spec.stage_buf;
    } else {
      stage_hold = -1;
      L = stage_begin(std::max(nent, 1));
    }
    if (t0 > 0 && !spec_layout) {
      // the speculation staged its clusters for a different layout: stage them again
      pool_for(t0, [&](int t) { stage_entry(L, full ? touched[t] : t, touched[t]); });
    }
    int berr = 0, gsl_t = -1;
    if (t0 < T) {
      pj_setup(touched, t0, h_counts.data(), h_freq.p, h_center.data(), h_sigma.data(), L, full, nullptr, false);
      pj_launch();
      berr = pj_finish();
      gsl_t = pj.gsl.load();
      mark("B+C");
    }
    sa.finish();                                      // the host stream continues after the draws
    phi_prefetch = std::max<int64_t>(4096, sa.used + sa.used / 4 + 512);
    sa.n = 0;                                         // consumed
    if (berr) { err = "center draw failed"; return berr; }
    if (gsl_t >= 0) { err = "norm_const2 - hypergeometric diverging with infinity"; return kGsl; }
    if (full) {
      // labels that were not updated still need their (unchanged) tables staged
      std::vector<char> done(K, 0);
      for (int k : touched) done[k] = 1;
      for (int k = 0; k < K; ++k)
        if (!done[k]) stage_entry(L, k, k);
      if (K && defer_commit && spec_layout) {
        // committed by flush_commit, after the next speculative update_phi is started
        commit_later.active = true;
        commit_later.dev = false;
        commit_later.buf = stage_fill;
        commit_later.nent = K;
        stage_hold = stage_fill;
      } else if (K) {
        stage_commit(L, K, true);
      }
      tables_dirty = false;
    } else if (T) {
      stage_commit(L, T, false);
    }
    auto t2 = std::chrono::steady_clock::now();
    mark("commit");
    stats.t_stats_ms += std::chrono::duration<double, std::milli>(t1 - t0c).count();
    stats.t_host_phi_ms += std::chrono::duration<double, std::milli>(t2 - t1).count();
    return kOk;
  }

  // ------------------------------------------------------------------ loglik
  int compute_loglikelihood(double* out) {
    if (!have_state) { err = "no state"; return kArg; }
    if (dev_ll_version == labels_version && !tables_dirty && !(debug & 4)) {
      // the full device update_phi of these labels summed the regrouped terms (phi.hip)
      *out = dev_ll;
      return kOk;
    }
    if (tables_dirty) upload_clusters();
    if (freq_version == labels_version && stage_full && !(debug & 4)) {
      // the labels have not moved since the last full histogram: the sum over points
      // regroups exactly into per-(cluster, attribute) match / mismatch counts times the
      // dhamming table values (the tables of the last full upload, still in h_stage)
      auto t0 = std::chrono::steady_clock::now();
      const UploadLayout L = upload_layout(K, dp, d, bw);
      const double* tab = (const double*)(h_stage_buf[stage_last].p + L.off_tab);
      double hi = 0.0, lo = 0.0;
      auto add = [&](double a) {
        const double s = hi + a, bb = s - hi;
        lo += (hi - (s - bb)) + (a - bb);
        hi = s;
      };
      for (int k = 0; k < K; ++k) {
        const double nk = (double)h_counts[k];
        for (int j = 0; j < d; ++j) {
          const double match = (double)h_freq.p[((size_t)k * d + j) * mmax + (h_center[(size_t)k * d + j] - 1)];
          add(match * tab[((size_t)k * d + j) * 2]);
          add((nk - match) * tab[((size_t)k * d + j) * 2 + 1]);
        }
      }
      *out = hi + lo;
      stats.t_loglik_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      return kOk;
    }
    HIPCHK(hipEventRecord(ev[3], stream));
    const int nb = (n + kBlock - 1) / kBlock;
    d_partial.ensure((size_t)2 * nb);
    LoglikArgs la;
    la.codes_t = d_codes_t.p; la.n = n; la.d = d; la.nq = nq; la.label = d_c.p;
    la.cl = ParamTables{d_slot_codes.p, d_slot_tab.p};
    la.partial = d_partial.p;
    HIPCHK(launch_loglik(la, stream));
    h_partial.ensure((size_t)2 * nb);
    HIPCHK(hipMemcpyAsync(h_partial.p, d_partial.p, (size_t)2 * nb * 8, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipEventRecord(ev[4], stream));
    HIPCHK(hipStreamSynchronize(stream));
    float t = 0;
    HIPCHK(hipEventElapsedTime(&t, ev[3], ev[4]));
    stats.t_loglik_ms += t;
    double hi = 0.0, lo = 0.0;
    for (int b = 0; b < nb; ++b) {
      const double a = h_partial.p[2 * b];
      const double s = hi + a, bb = s - hi;
      lo += (hi - (s - bb)) + (a - bb) + h_partial.p[2 * b + 1];
      hi = s;
    }
    *out = hi + lo;
    return kOk;
  }

  int loglik_matrix(double* L, int32_t* H) {
    if (!have_state) { err = "no state"; return kArg; }
    if (tables_dirty) upload_clusters();
    DevBuf<double> dl;
    DevBuf<int> dh;
    dl.ensure((size_t)K * n);
    dh.ensure((size_t)K * n);
    HIPCHK(launch_lmatrix(d_codes_t.p, n, d, nq, ParamTables{d_slot_codes.p, d_slot_tab.p}, K, dl.p, dh.p, n,
                          stream));
    std::vector<double> tl((size_t)K * n);
    std::vector<int> th((size_t)K * n);
    HIPCHK(hipMemcpyAsync(tl.data(), dl.p, tl.size() * 8, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipMemcpyAsync(th.data(), dh.p, th.size() * 4, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < K; ++k) {
        if (L) L[(size_t)i * K + k] = tl[(size_t)k * n + i];
        if (H) H[(size_t)i * K + k] = th[(size_t)k * n + i];
      }
    return kOk;
  }

  // ------------------------------------------------------------------ chain driver
  int run_markov_chain(const hdpm_chain_params* p, const int32_t* c_init, int32_t* o_tot, int32_t* o_c,
                       double* o_ll, int32_t* o_acc, int32_t* o_final, double* o_time);
  int split_and_merge(int t, int r, int idx_1_sm, int* accepted);
  int init_chain(const hdpm_chain_params* p, const int32_t* c_init);
  int iteration(const hdpm_chain_params* p, int iter, int* idx_1_sm, int* accepted, double* ll,
                bool launch_next = false, int32_t* labels_out = nullptr);
};

}  // namespace hdpm

#include "split_merge.inl"

namespace hdpm {

// la:27-77
int Ctx::init_chain(const hdpm_chain_params* p, const int32_t* c_init) {
  if (!n) { err = "set_data first"; return kArg; }
  rng_sync();
  K = p->L;
  h_c.resize(n);
  if (c_init) {
    int mn = c_init[0];
    for (int i = 1; i < n; ++i) mn = std::min(mn, (int)c_init[i]);
    for (int i = 0; i < n; ++i) h_c[i] = c_init[i] - mn;
    int mx = *std::max_element(h_c.begin(), h_c.end());
    std::vector<char> seen(mx + 1, 0);
    int u = 0;
    for (int i = 0; i < n; ++i) if (!seen[h_c[i]]) { seen[h_c[i]] = 1; u++; }
    K = u;
    if (mx >= K) { err = "initial labels must be contiguous after subtracting the minimum"; return kArg; }
  } else {
    if (p->L <= 0) { err = "L must be positive for a random initial assignment"; return kArg; }
    for (int i = 0; i < n; ++i) h_c[i] = (int)(p->L * rng.unif() + 1) - 1;
  }
  // la:46-48: all centers, then all sigmas
  h_center.assign((size_t)K * d, 0);
  h_sigma.assign((size_t)K * d, 0.0);
  for (int k = 0; k < K; ++k) sample_center_uniform(&h_center[(size_t)k * d]);
  for (int k = 0; k < K; ++k) {
    int st = sample_sigma(v.data(), w.data(), &h_sigma[(size_t)k * d]);
    if (st) { err = "rhig failed"; return st; }
  }
  recount();
  upload_labels();
  upload_clusters();
  have_state = true;
  int st = update_phi(nullptr, 0);  // la:51
  if (st) return st;
  return generate_pool((int64_t)n * p->m * p->thinning);  // la:67-77
}

// la:85-132, one iteration
int Ctx::iteration(const hdpm_chain_params* p, int iter, int* idx_1_sm, int* accepted, double* ll, bool launch_next,
                   int32_t* labels_out) {
  int st;
  *accepted = 0;
  trace.clear();
  mark("start");
  const bool n8 = p->neal8 && iter % p->n8_step_size == 0;
  const bool sm_now = p->split_merge && iter % p->sam_step_size == 0;
  const bool next_n8 = p->neal8 && (iter + 1) % p->n8_step_size == 0;
  // the next iteration's speculative update_phi started before this one's tables are
  // committed and its log-likelihood summed (both off the host's critical path, which is the
  // chain of update_phi draws): when this iteration is a lone Neal-8 sweep whose update
  // came from the speculation and whose log-likelihood needs no device work
  const bool early = n8 && !sm_now && next_n8 && iter % 1000 != 0 && !(debug & 2097152);
  if (!n8) cancel_ahead();
  if (n8) {                                              // la:94-103
    // the next sweep may be enqueued while this one's update is drawn (pre_enqueue)
    deep_ok = early && launch_next && !(debug & 4194304);
    st = neal8_sweep(p->m);
    deep_ok = false;
    if (st) {
      pre_release();
      return st;
    }
    // a recorded iteration's labels, before a sweep enqueued ahead can be given the go
    if (labels_out) capture_labels();
    defer_commit = early;
    st = update_phi(nullptr, 0);
    defer_commit = false;
    if (st) {
      pre_release();
      flush_commit();
      return st;
    }
  }
  bool prepared = false;
  if (pre.active) {
    if (early && launch_next && pipe_go(p->m)) prepared = true;
    else pre_release();
  }
  if (!prepared && early && commit_later.active && freq_version == labels_version && !(debug & 4) && !tables_dirty) {
    prepare_next_sweep(p->m, launch_next);               // spec_launch, flush_commit, round 0
    prepared = true;
  }
  flush_commit();
  if (sm_now) {                                          // la:111-115
    const auto t0 = std::chrono::steady_clock::now();
    st = split_and_merge(p->t, p->r, *idx_1_sm, accepted);
    stats.t_sm_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    stats.sm_moves++;
    if (st) return st;
    *idx_1_sm = (*idx_1_sm + 1) % n;
  }
  if (iter % 1000 == 0) {                                // la:123-129
    st = generate_pool((int64_t)n * p->m * p->thinning);
    if (st) return st;
  }
  st = compute_loglikelihood(ll);                        // la:132
  mark("loglik");
  if (!st && labels_out) {                               // la:145 (before the next sweep is launched)
    if (sm_now || !n8) capture_labels();                 // (split-merge may have relabelled)
    std::memcpy(labels_out, h_c.data(), (size_t)n * 4);
  }
  // the next iteration starts with a sweep: prepare it now (cancelled by any other call;
  // launched on the device too when the caller runs that iteration next, launch_next)
  if (!st && next_n8 && !prepared) {
    prepare_next_sweep(p->m, launch_next);
    prepared = true;
  }
  if (prepared && ahead.active && host_spec()) phi_lookahead();
  mark("ahead");
  if ((debug & 32) && trace.size() > 1) {
    if (trace_alloc0 < 0) trace_alloc0 = g_dev_allocs.load();
    for (size_t k = 1; k < trace.size(); ++k) {
      const double us = std::chrono::duration<double, std::micro>(trace[k].second - trace[k - 1].second).count();
      trace_add(trace[k].first, us);
    }
    const double tot = std::chrono::duration<double, std::micro>(trace.back().second - trace.front().second).count();
    trace_add("total", tot);
    if (tot > 180.0 && trace_slow++ < 12) {              // the segments of a slow iteration
      std::string line = "[slow iteration " + std::to_string(trace_iters) + "]";
      for (size_t k = 1; k < trace.size(); ++k) {
        char buf[64];
        std::snprintf(buf, sizeof(buf), " %s %.0f", trace[k].first,
                      std::chrono::duration<double, std::micro>(trace[k].second - trace[k - 1].second).count());
        line += buf;
      }
      std::fprintf(stderr, "%s%s\n", line.c_str(), spec_line);
    }
    trace_iters++;
  }
  if ((debug & 2) && trace.size() > 1) {
    std::string line = "[iter]";
    for (size_t k = 1; k < trace.size(); ++k) {
      char buf[96];
      std::snprintf(buf, sizeof(buf), " %s %.1f", trace[k].first,
                    std::chrono::duration<double, std::micro>(trace[k].second - trace[k - 1].second).count());
      line += buf;
    }
    std::fprintf(stderr, "%s us\n", line.c_str());
  }
  return st;
}

// la:6-174
int Ctx::run_markov_chain(const hdpm_chain_params* p, const int32_t* c_init, int32_t* o_tot, int32_t* o_c,
                          double* o_ll, int32_t* o_acc, int32_t* o_final, double* o_time) {
  int st = init_chain(p, c_init);
  if (st) return st;
  auto t0 = std::chrono::steady_clock::now();
  int idx_1_sm = 0;
  const int total = (p->iterations + p->burnin) * p->thinning;
  for (int iter = 0; iter < total; ++iter) {
    int accepted = 0;
    double ll = 0.0;
    const bool rec = iter >= p->thinning * p->burnin && iter % p->thinning == 0;   // la:140-153
    const int at = rec ? iter / p->thinning - p->burnin : 0;
    st = iteration(p, iter, &idx_1_sm, &accepted, &ll, iter + 1 < total, (rec && o_c) ? o_c + (size_t)at * n : nullptr);
    if (st) return st;
    if (rec) {
      if (o_tot) o_tot[at] = K;
      if (o_ll) o_ll[at] = ll;
      if (o_acc) o_acc[at] = accepted;
    }
  }
  if (o_final) {
    download_labels();
    std::memcpy(o_final, h_c.data(), (size_t)n * 4);
  }
  if (o_time) o_time[0] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return kOk;
}

}  // namespace hdpm

// ====================================================================== C ABI
using hdpm::Ctx;
using hdpm::HipError;
using hdpm::ScopedPin;
using hdpm::DevBuf;

#define GUARD(body)                                                            \
  try {                                                                        \
    body                                                                       \
  } catch (const hdpm::HipError& he) {                                         \
    ctx->err = std::string("HIP error: ") + hipGetErrorString(he.e) + " at " + he.what; \
    return HDPM_E_DEVICE;                                                      \
  } catch (const std::bad_alloc&) {                                            \
    ctx->err = "host allocation failed";                                       \
    return HDPM_E_ARG;                                                         \
  } catch (...) {                                                              \
    ctx->err = "unknown exception";                                            \
    return HDPM_E_ARG;                                                         \
  }

extern "C" {

int hdpm_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

int hdpm_ctx_create(int32_t device, hdpm_ctx** out) {
  if (!out) return HDPM_E_ARG;
  *out = nullptr;
  int cnt = 0;
  if (hipGetDeviceCount(&cnt) != hipSuccess || cnt <= device || device < 0) return HDPM_E_NODEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return HDPM_E_NODEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return HDPM_E_NODEVICE;
  auto* c = new (std::nothrow) Ctx();
  if (!c) return HDPM_E_ARG;
  c->device = device;
  // the host pool homed next to this GPU: one pool per home domain, so contexts on GPUs with
  // different homes in one process (an R session with replicas on two GPUs) do not share one
  try {
    c->hpool = &hdpm::HostPool::for_home(hdpm::gpu_home_domain(device));
  } catch (...) {
    delete c;
    return HDPM_E_ARG;
  }
  // the sweep's stream at the highest priority, the generator windows' side stream at the
  // lowest: a window's generation (~1 ms per 16 sweeps of draws) then takes the CUs the
  // sweep leaves (HDPM_STREAM_PRIO=0: default priorities)
  int prio_lo = 0, prio_hi = 0;
  const char* sp = std::getenv("HDPM_STREAM_PRIO");
  if (!(sp && sp[0] == '0') && hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_lo = prio_hi = 0;
  // (testing, HDPM_STREAM_PRIO=2: the sweep's stream at the generator's priority, the device
  // update_phi's above it)
  const int prio_sweep = (sp && sp[0] == '2') ? prio_lo : prio_hi;
  if (std::getenv("HDPM_PHI_TRACE")) std::fprintf(stderr, "[streams] priorities %d..%d sweep %d\n", prio_lo, prio_hi, prio_sweep);
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_sweep) != hipSuccess) {
    delete c;
    return HDPM_E_DEVICE;
  }
  for (auto& e : c->ev) (void)hipEventCreate(&e);
  if (hipStreamCreateWithPriority(&c->gstream, hipStreamNonBlocking, prio_lo) != hipSuccess) {
    delete c;
    return HDPM_E_DEVICE;
  }
  if (hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return HDPM_E_DEVICE;
  }
  // the speculative device update_phi at the sweep's priority (it runs beside the sweep)
  if (hipStreamCreateWithPriority(&c->pstream, hipStreamNonBlocking, prio_hi) != hipSuccess) {
    delete c;
    return HDPM_E_DEVICE;
  }
  c->rng.set_seed(0);
  *out = reinterpret_cast<hdpm_ctx*>(c);
  return HDPM_OK;
}

void hdpm_ctx_destroy(hdpm_ctx* h) {
  auto* c = reinterpret_cast<Ctx*>(h);
  if (!c) return;
  (void)hipSetDevice(c->device);
  delete c;
}

const char* hdpm_last_error(const hdpm_ctx* h) {
  auto* c = reinterpret_cast<const Ctx*>(h);
  return c ? c->err.c_str() : "null context";
}

#define CTX_KEEP()                              \
  auto* ctx = reinterpret_cast<Ctx*>(h);        \
  if (!ctx) return HDPM_E_ARG;                  \
  hdpm::PoolScope pool_scope_(ctx->hpool);      \
  (void)hipSetDevice(ctx->device);              \
  ctx->err.clear();
// every entry point but the sweep and the iteration drops a prepared sweep first
#define CTX()                                   \
  CTX_KEEP();                                   \
  GUARD(ctx->cancel_ahead();)

int hdpm_set_data(hdpm_ctx* h, const uint8_t* codes, int32_t n, int32_t d, const int32_t* attrisize, double gamma,
                  const double* v, const double* w) {
  CTX();
  if (!codes || !attrisize || !v || !w) return HDPM_E_ARG;
  GUARD(return ctx->set_data(codes, n, d, attrisize, gamma, v, w);)
}

int hdpm_rng_set_seed(hdpm_ctx* h, uint32_t seed) {
  CTX();
  ctx->rng_drop_pending();
  ctx->rng.set_seed(seed);
  return HDPM_OK;
}
int hdpm_rng_set_state(hdpm_ctx* h, const int32_t* s) {
  CTX();
  if (!s) return HDPM_E_ARG;
  ctx->rng_drop_pending();
  ctx->rng.import625(s);
  return HDPM_OK;
}
int hdpm_rng_get_state(const hdpm_ctx* h, int32_t* s) {
  // the state is logically const; an adoption still in flight lands first
  auto* ctx = const_cast<Ctx*>(reinterpret_cast<const Ctx*>(h));
  if (!ctx || !s) return HDPM_E_ARG;
  hdpm::PoolScope pool_scope_(ctx->hpool);
  GUARD({
    ctx->cancel_ahead();
    ctx->rng_sync();
    ctx->rng.export625(s);
    return HDPM_OK;
  })
}

int hdpm_set_state(hdpm_ctx* h, const int32_t* c_i, int32_t K, const double* centers, const double* sigma) {
  CTX();
  if (!c_i || (K > 0 && (!centers || !sigma))) return HDPM_E_ARG;
  GUARD(return ctx->set_state(c_i, K, centers, sigma);)
}
int hdpm_get_state(hdpm_ctx* h, int32_t* c_i, int32_t* K, double* centers, double* sigma, int32_t cap) {
  CTX();
  GUARD(return ctx->get_state(c_i, K, centers, sigma, cap);)
}
int hdpm_set_pool(hdpm_ctx* h, const double* centers, const double* sigma, int64_t P) {
  CTX();
  if (!centers || !sigma) return HDPM_E_ARG;
  GUARD(return ctx->set_pool(centers, sigma, P);)
}
int hdpm_get_pool(hdpm_ctx* h, double* centers, double* sigma, int64_t P) {
  CTX();
  if (P != ctx->P) { ctx->err = "pool size mismatch"; return HDPM_E_ARG; }
  GUARD(ctx->get_pool(centers, sigma);)
  return HDPM_OK;
}
int hdpm_generate_pool(hdpm_ctx* h, int64_t P) {
  CTX();
  GUARD(return ctx->generate_pool(P);)
}
int hdpm_neal8_sweep(hdpm_ctx* h, int32_t m) {
  CTX_KEEP();
  ScopedPin pin;
  GUARD(return ctx->neal8_sweep(m);)
}
int hdpm_update_phi(hdpm_ctx* h, const int32_t* idx, int32_t n_idx) {
  CTX();
  ScopedPin pin;
  if (n_idx > 0 && !idx) return HDPM_E_ARG;
  GUARD(return ctx->update_phi(idx, n_idx);)
}
int hdpm_compute_loglikelihood(hdpm_ctx* h, double* out) {
  CTX();
  if (!out) return HDPM_E_ARG;
  GUARD(return ctx->compute_loglikelihood(out);)
}
int hdpm_loglik_matrix(hdpm_ctx* h, double* L, int32_t* H) {
  CTX();
  GUARD(return ctx->loglik_matrix(L, H);)
}
int hdpm_restricted_gibbs(hdpm_ctx* h, const int32_t* S, int32_t nS, int32_t i1, int32_t i2, int32_t t) {
  CTX();
  GUARD(return hdpm::sm_restricted_gibbs_device(ctx, S, nS, i1, i2, t);)
}
int hdpm_logprobgs_c_i(hdpm_ctx* h, const int32_t* g_c_i, const int32_t* S, int32_t nS, int32_t i1, int32_t i2,
                       double* out) {
  CTX();
  GUARD(return hdpm::sm_logprobgs_c_i_api(ctx, g_c_i, S, nS, i1, i2, out);)
}
int hdpm_split_and_merge(hdpm_ctx* h, int32_t t, int32_t r, int32_t idx_1_sm, int32_t* accepted) {
  CTX();
  ScopedPin pin;
  int acc = 0;
  int st;
  GUARD(st = ctx->split_and_merge(t, r, idx_1_sm, &acc);)
  if (accepted) *accepted = acc;
  return st;
}
int hdpm_run_markov_chain(hdpm_ctx* h, const hdpm_chain_params* p, const int32_t* c_i_init, int32_t* out_total_cls,
                          int32_t* out_c_i, double* out_loglik, int32_t* out_accepted, int32_t* final_ass,
                          double* out_time_s) {
  CTX();
  if (!p) return HDPM_E_ARG;
  ScopedPin pin;
  GUARD(return ctx->run_markov_chain(p, c_i_init, out_total_cls, out_c_i, out_loglik, out_accepted, final_ass,
                                     out_time_s);)
}
int hdpm_init_chain(hdpm_ctx* h, const hdpm_chain_params* p, const int32_t* c_i_init) {
  CTX();
  ScopedPin pin;
  if (!p) return HDPM_E_ARG;
  GUARD(return ctx->init_chain(p, c_i_init);)
}
int hdpm_iteration(hdpm_ctx* h, const hdpm_chain_params* p, int32_t iter, int32_t* idx_1_sm, int32_t* accepted,
                   double* loglik) {
  CTX_KEEP();
  if (!p || !idx_1_sm) return HDPM_E_ARG;
  ScopedPin pin;
  int acc = 0;
  double ll = 0.0;
  int st;
  GUARD(st = ctx->iteration(p, iter, idx_1_sm, &acc, &ll);)
  if (accepted) *accepted = acc;
  if (loglik) *loglik = ll;
  return st;
}
int hdpm_iterations(hdpm_ctx* h, const hdpm_chain_params* p, int32_t iter0, int32_t count, int32_t* idx_1_sm,
                    int32_t* accepted, double* loglik) {
  CTX_KEEP();
  if (!p || !idx_1_sm || count < 0) return HDPM_E_ARG;
  ScopedPin pin;
  int st = HDPM_OK;
  GUARD({
    for (int k = 0; k < count && st == HDPM_OK; ++k) {
      int acc = 0;
      double ll = 0.0;
      st = ctx->iteration(p, iter0 + k, idx_1_sm, &acc, &ll, k + 1 < count);
      if (accepted) accepted[k] = acc;
      if (loglik) loglik[k] = ll;
    }
  })
  return st;
}
int hdpm_iterations_record(hdpm_ctx* h, const hdpm_chain_params* p, int32_t iter0, int32_t count, int32_t* idx_1_sm,
                           int32_t* accepted, double* loglik, int32_t* total_cls, int32_t* c_i, int32_t* nsaved) {
  CTX_KEEP();
  if (!p || !idx_1_sm || count < 0 || p->thinning < 1) return HDPM_E_ARG;
  ScopedPin pin;
  int st = HDPM_OK;
  int saved = 0;
  GUARD({
    for (int k = 0; k < count && st == HDPM_OK; ++k) {
      const int iter = iter0 + k;
      const bool rec = iter >= p->thinning * p->burnin && iter % p->thinning == 0;   // la:140
      int acc = 0;
      double ll = 0.0;
      st = ctx->iteration(p, iter, idx_1_sm, &acc, &ll, k + 1 < count,
                          rec && c_i ? c_i + (size_t)saved * ctx->n : nullptr);
      if (accepted) accepted[k] = acc;
      if (loglik) loglik[k] = ll;
      if (st == HDPM_OK && rec) {                                            // la:141-153
        if (total_cls) total_cls[saved] = ctx->K;
        ctx->record_params();
        saved++;
      }
    }
  })
  if (nsaved) *nsaved = saved;
  return st;
}
int hdpm_record_take(hdpm_ctx* h, double* centers, double* sigmas, int64_t* nrows) {
  CTX_KEEP();
  if (!nrows) return HDPM_E_ARG;
  const int64_t rows = ctx->d ? (int64_t)(ctx->rec_cen.size() / (size_t)ctx->d) : 0;
  *nrows = rows;
  if (!centers || !sigmas) return HDPM_OK;
  for (size_t q = 0; q < ctx->rec_cen.size(); ++q) centers[q] = (double)ctx->rec_cen[q];
  std::memcpy(sigmas, ctx->rec_sig.data(), ctx->rec_sig.size() * 8);
  ctx->rec_cen.clear();
  ctx->rec_sig.clear();
  return HDPM_OK;
}
int hdpm_rng_fill_device(hdpm_ctx* h, int64_t count, uint32_t* out) {
  CTX();
  if (count <= 0 || !out) return HDPM_E_ARG;
  GUARD({
    const uint32_t* p = ctx->device_draws(count);
    HIPCHK(hipMemcpyAsync(out, p, (size_t)count * 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return HDPM_OK;
  })
}
int hdpm_get_stats(const hdpm_ctx* h, hdpm_stats* out) {
  auto* ctx = reinterpret_cast<const Ctx*>(h);
  if (!ctx || !out) return HDPM_E_ARG;
  *out = ctx->stats;
  return HDPM_OK;
}
// Counters and synchronisation leave a prepared sweep in place (they change no chain
// state), so a caller that runs hdpm_iterations in batches keeps the pipeline warm across
// them; changing the debug mode drops it (the prepared work followed the old mode).
int hdpm_reset_stats(hdpm_ctx* h) {
  CTX_KEEP();
  ctx->stats = hdpm_stats{};
  return HDPM_OK;
}
int hdpm_set_debug(hdpm_ctx* h, int32_t mode) {
  CTX_KEEP();
  if (mode != ctx->debug) GUARD(ctx->cancel_ahead();)
  ctx->debug = mode;
  return HDPM_OK;
}
int hdpm_get_pool_heads(hdpm_ctx* h, uint64_t* out, int64_t P) {
  CTX();
  if (!out || P != ctx->P || P <= 0) { ctx->err = "pool size mismatch"; return HDPM_E_ARG; }
  if (!hdpm::head_fits(ctx->wb, ctx->Ws)) { ctx->err = "no pool-entry heads for this layout"; return HDPM_E_ARG; }
  GUARD({
    HIPCHK(hipMemcpyAsync(out, ctx->d_pool_head.p, (size_t)P * hdpm::head_stride(ctx->wb, ctx->Ws) * 8, hipMemcpyDeviceToHost,
                          ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return HDPM_OK;
  })
}
int hdpm_get_option(hdpm_ctx* h, int32_t option, double* value) {
  CTX();
  if (!value) return HDPM_E_ARG;
  switch (option) {
    case HDPM_OPT_HIG_LOGSPACE: *value = ctx->hig_log ? 1.0 : 0.0; return HDPM_OK;
    case HDPM_OPT_PHI_DEVICE: *value = (double)ctx->phi_mode; return HDPM_OK;
    case HDPM_OPT_PIPE_WAIT_US: *value = (double)ctx->pipe_limit_ticks * 0.01 * (ctx->pipe_host_check ? 1 : -1); return HDPM_OK;
    case HDPM_OPT_FPG_WAIT_US: *value = (double)ctx->fpg_limit_ticks * 0.01; return HDPM_OK;
    case HDPM_OPT_FPG_FAIL_AT: *value = (double)ctx->fpg_fail_at; return HDPM_OK;
    case HDPM_OPT_EXACT_KERNEL: *value = (double)ctx->exact_pref; return HDPM_OK;
    case HDPM_OPT_LAT_NEGLIGIBLE: *value = ctx->lat_negl; return HDPM_OK;
    case HDPM_OPT_SM_WIDE_WAIT_US: *value = (double)ctx->sm_wide_ticks * 0.01; return HDPM_OK;
    case HDPM_OPT_SM_CHAIN: *value = (double)ctx->sm_chain_mode; return HDPM_OK;
    default:
      ctx->err = "unknown option";
      return HDPM_E_ARG;
  }
}
int hdpm_set_option(hdpm_ctx* h, int32_t option, double value) {
  CTX();
  switch (option) {
    case HDPM_OPT_HIG_LOGSPACE:
      ctx->hig_log = value != 0.0;
      return HDPM_OK;
    case HDPM_OPT_PHI_DEVICE:
      if (!(value == 0.0 || value == 1.0 || value == 2.0 || value == 3.0)) {
        ctx->err = "phi device: 0 host, 1 device, 2 device (general kernels), 3 automatic";
        return HDPM_E_ARG;
      }
      GUARD(ctx->cancel_ahead();)
      ctx->phi_mode = (int)value;
      return HDPM_OK;
    case HDPM_OPT_FPG_WAIT_US:
      if (!(value > 0.0) || !std::isfinite(value)) { ctx->err = "fpg wait limit must be positive"; return HDPM_E_ARG; }
      GUARD(ctx->cancel_ahead();)
      ctx->fpg_limit_ticks = std::max(1LL, (long long)(value * 100.0));
      return HDPM_OK;
    case HDPM_OPT_FPG_FAIL_AT:
      if (value < 0.0 || value > 1e9) { ctx->err = "fpg fail ordinal out of range"; return HDPM_E_ARG; }
      GUARD(ctx->cancel_ahead();)
      ctx->fpg_fail_at = (int)value;
      return HDPM_OK;
    case HDPM_OPT_EXACT_KERNEL:
      if (value < 0.0 || value > 3.0) { ctx->err = "exact kernel: 0 auto, 1 mass, 2 lanes, 3 level tables"; return HDPM_E_ARG; }
      GUARD(ctx->cancel_ahead();)
      ctx->exact_pref = (int)value;
      return HDPM_OK;
    case HDPM_OPT_LAT_NEGLIGIBLE:
      if (!(value >= 40.0)) { ctx->err = "latent negligibility margin must be >= 40"; return HDPM_E_ARG; }
      GUARD(ctx->cancel_ahead();)
      ctx->lat_negl = value;
      return HDPM_OK;
    case HDPM_OPT_SM_WIDE_WAIT_US:
      if (!(value >= 0.0) || !(value <= 1e9)) { ctx->err = "wide scan wait must be in [0, 1e9] us"; return HDPM_E_ARG; }
      GUARD(ctx->cancel_ahead();)
      ctx->sm_wide_ticks = (long long)(value * 100.0);   // 0: every wide scan gives up at its first barrier
      return HDPM_OK;
    case HDPM_OPT_SM_CHAIN:
      if (!(value >= 0.0) || !(value <= 1000.0) || value != std::floor(value)) {
        ctx->err = "sm chain: 0 off, 1 on, 2 + 3k / 3 + 3k / 4 + 3k stop at scan k / its updates (testing)";
        return HDPM_E_ARG;
      }
      GUARD(ctx->cancel_ahead();)
      ctx->sm_chain_mode = (int)value;
      return HDPM_OK;
    case HDPM_OPT_PIPE_WAIT_US:
      if (value == 0.0 || !std::isfinite(value)) { ctx->err = "pipe wait limit must be non-zero"; return HDPM_E_ARG; }
      GUARD(ctx->cancel_ahead();)
      ctx->pipe_limit_ticks = std::max(1LL, (long long)(std::fabs(value) * 100.0));
      ctx->pipe_host_check = value > 0;
      return HDPM_OK;
    default:
      ctx->err = "unknown option";
      return HDPM_E_ARG;
  }
}
int hdpm_psm_build(hdpm_ctx* h, const int32_t* c_trace, int32_t M, int32_t N) {
  CTX();
  if (!c_trace || M <= 0 || N <= 0) return HDPM_E_ARG;
  for (int64_t q = 0; q < (int64_t)M * N; ++q)
    if (c_trace[q] < 0 || c_trace[q] > 254) { ctx->err = "psm: labels must be in 0..254"; return HDPM_E_ARG; }
  GUARD({
    const int Mp = (M + 15) & ~15;
    ctx->d_psm_trace.ensure((size_t)M * N);
    ctx->d_psm_lab.ensure((size_t)N * Mp);
    ctx->d_psm_cnt.ensure((size_t)N * N);
    HIPCHK(hipMemcpyAsync(ctx->d_psm_trace.p, c_trace, (size_t)M * N * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hdpm::launch_psm(ctx->d_psm_trace.p, M, N, ctx->d_psm_lab.p, ctx->d_psm_cnt.p, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    ctx->psm_N = N;
    ctx->psm_M = M;
    return HDPM_OK;
  })
}
int hdpm_psm_rows(hdpm_ctx* h, int32_t row0, int32_t nrows, double* out) {
  CTX();
  const int N = ctx->psm_N;
  if (!out || N == 0 || row0 < 0 || nrows < 0 || row0 + nrows > N) return HDPM_E_ARG;
  GUARD({
    std::vector<uint32_t> c((size_t)nrows * N);
    HIPCHK(hipMemcpyAsync(c.data(), ctx->d_psm_cnt.p + (size_t)row0 * N, c.size() * 4, hipMemcpyDeviceToHost,
                          ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    const double M = (double)ctx->psm_M;
    for (size_t q = 0; q < c.size(); ++q) out[q] = (double)c[q] / M;
    return HDPM_OK;
  })
}
int hdpm_psm_vi_lb(hdpm_ctx* h, const int32_t* cls, int32_t ncand, double* out) {
  CTX();
  const int N = ctx->psm_N;
  if (!cls || !out || N == 0 || ncand <= 0) return HDPM_E_ARG;
  GUARD({
    ctx->d_psm_cls.ensure((size_t)ncand * N);
    ctx->d_psm_all.ensure((size_t)N);
    ctx->d_psm_same.ensure((size_t)ncand * N);
    HIPCHK(hipMemcpyAsync(ctx->d_psm_cls.p, cls, (size_t)ncand * N * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hdpm::launch_vi_terms(ctx->d_psm_cnt.p, N, ctx->psm_M, ctx->d_psm_cls.p, ncand, ctx->d_psm_all.p,
                                 ctx->d_psm_same.p, ctx->stream));
    std::vector<double> all((size_t)N);
    std::vector<double> same((size_t)ncand * N);
    HIPCHK(hipMemcpyAsync(all.data(), ctx->d_psm_all.p, all.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipMemcpyAsync(same.data(), ctx->d_psm_same.p, same.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    // mcclust.ext VI.lb: f = sum_i (log2 n_{c_i} + log2 sum_j psm_ij - 2 log2 sum_{j in c_i} psm_ij) / n
    std::vector<int> sz;
    for (int c = 0; c < ncand; ++c) {
      const int32_t* cl = cls + (size_t)c * N;
      int mx = 0;
      for (int i = 0; i < N; ++i) mx = std::max(mx, cl[i]);
      sz.assign((size_t)mx + 1, 0);
      for (int i = 0; i < N; ++i) {
        if (cl[i] < 0) { ctx->err = "psm: negative cluster label"; return HDPM_E_ARG; }
        sz[cl[i]]++;
      }
      double f = 0.0;
      for (int i = 0; i < N; ++i)
        f = f + (std::log2((double)sz[cl[i]]) + std::log2(all[i]) - 2 * std::log2(same[(size_t)c * N + i])) / N;
      out[c] = f;
    }
    return HDPM_OK;
  })
}
int hdpm_debug_draw(hdpm_ctx* h, const double* logw, int32_t E, double rU, int32_t two_way, int32_t ocml,
                    int32_t* pick) {
  CTX();
  if (!logw || !pick || E < 1 || E > 256 || (two_way && E != 2)) return HDPM_E_ARG;
  GUARD({
    DevBuf<double> dw;
    DevBuf<int> dp;
    dw.ensure((size_t)E);
    dp.ensure(1);
    HIPCHK(hipMemcpyAsync(dw.p, logw, (size_t)E * 8, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hdpm::launch_debug_draw(dw.p, E, rU, two_way, ocml, dp.p, ctx->stream));
    HIPCHK(hipMemcpyAsync(pick, dp.p, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return HDPM_OK;
  })
}
int hdpm_debug_math(hdpm_ctx* h, const double* x, int64_t n, int32_t fn, int32_t ocml, double* out) {
  CTX();
  if (!x || !out || n <= 0 || (fn != 0 && fn != 1)) return HDPM_E_ARG;
  GUARD({
    DevBuf<double> dx;
    DevBuf<double> dy;
    dx.ensure((size_t)n);
    dy.ensure((size_t)n);
    HIPCHK(hipMemcpyAsync(dx.p, x, (size_t)n * 8, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hdpm::launch_debug_math(dx.p, n, fn, ocml, dy.p, ctx->stream));
    HIPCHK(hipMemcpyAsync(out, dy.p, (size_t)n * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    return HDPM_OK;
  })
}
int hdpm_drop_prepared(hdpm_ctx* h) {
  CTX();
  return HDPM_OK;
}
int hdpm_synchronize(hdpm_ctx* h) {
  CTX_KEEP();
  // everything queued on the device, a prepared sweep's prefix included (a timed window
  // that ends here ends drained); the prepared sweep stays
  return hipStreamSynchronize(ctx->stream) == hipSuccess ? HDPM_OK : HDPM_E_DEVICE;
}

}  // extern "C"
