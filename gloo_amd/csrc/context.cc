// context.cc -- see context.h.
#include "context.h"
#include "executor_internal.h"

#include <algorithm>

#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <chrono>
#include <cstdlib>
#include <thread>

#include "common.h"

namespace gloo {

// ---- ControlBlock ----------------------------------------------------------

ControlBlock::~ControlBlock() {
  if (base_ != nullptr) ::munmap(base_, kBytes);
  if (owner_ && !unlinked_ && !name_.empty()) ::shm_unlink(name_.c_str());
}

void ControlBlock::create(const std::string& name) {
  int fd = ::shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) GLX_THROW_IO("shm_open(", name, ") failed: ", strerror(errno));
  if (::ftruncate(fd, (off_t)kBytes) != 0) {
    int e = errno;
    ::close(fd);
    ::shm_unlink(name.c_str());
    GLX_THROW_IO("ftruncate(", name, ") failed: ", strerror(e));
  }
  void* p = ::mmap(nullptr, kBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) {
    ::shm_unlink(name.c_str());
    GLX_THROW_IO("mmap(", name, ") failed: ", strerror(errno));
  }
  base_ = static_cast<char*>(p);
  name_ = name;
  owner_ = true;
}

void ControlBlock::open(const std::string& name) {
  int fd = ::shm_open(name.c_str(), O_RDWR, 0600);
  if (fd < 0) GLX_THROW_IO("shm_open(", name, ") of a peer failed: ", strerror(errno));
  void* p = ::mmap(nullptr, kBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) GLX_THROW_IO("mmap(", name, ") of a peer failed: ", strerror(errno));
  base_ = static_cast<char*>(p);
  name_ = name;
  owner_ = false;
}

void ControlBlock::unlink() {
  if (owner_ && !unlinked_) {
    ::shm_unlink(name_.c_str());
    unlinked_ = true;
  }
}

uint32_t ControlBlock::allocWord() {
  std::lock_guard<std::mutex> g(m_);
  uint32_t w;
  if (!free_.empty()) {
    w = free_.back();
    free_.pop_back();
  } else {
    GLX_ENFORCE(next_ < kWords, "control block exhausted (", kWords, " words)");
    w = next_++;
  }
  word(w)->store(0, std::memory_order_release);
  return w;
}

void ControlBlock::freeWord(uint32_t i) {
  std::lock_guard<std::mutex> g(m_);
  free_.push_back(i);
}

// ---- Context -----------------------------------------------------------------

namespace {

std::atomic<uint64_t> g_ctx_counter{0};

void putStr(std::vector<char>& b, const std::string& s) {
  uint32_t n = (uint32_t)s.size();
  b.insert(b.end(), (char*)&n, (char*)&n + 4);
  b.insert(b.end(), s.begin(), s.end());
}

template <typename T>
void putPod(std::vector<char>& b, const T& v) {
  b.insert(b.end(), (const char*)&v, (const char*)&v + sizeof(T));
}

struct Reader {
  const std::vector<char>& b;
  size_t at = 0;
  template <typename T>
  T pod() {
    GLX_ENFORCE(at + sizeof(T) <= b.size(), "truncated endpoint record");
    T v;
    memcpy(&v, b.data() + at, sizeof(T));
    at += sizeof(T);
    return v;
  }
  std::string str() {
    uint32_t n = pod<uint32_t>();
    GLX_ENFORCE(at + n <= b.size(), "truncated endpoint record");
    std::string s(b.data() + at, b.data() + at + n);
    at += n;
    return s;
  }
};

std::string busIdOf(int device) {
  char buf[64] = {0};
  if (device >= 0 && hipDeviceGetPCIBusId(buf, sizeof(buf), device) == hipSuccess) {
    return std::string(buf);
  }
  return std::string();
}

}  // namespace

Context::Context(int rank_, int size_, int device) : rank(rank_), size(size_), device_(device) {
  GLX_ENFORCE(size_ >= 1, "context size must be >= 1, got ", size_);
  GLX_ENFORCE(rank_ >= 0 && rank_ < size_, "rank ", rank_, " out of range [0, ", size_, ")");
  if (device_ < 0) {
    int d = 0;
    if (hipGetDevice(&d) == hipSuccess) device_ = d;
  }
  peers_.resize(size_);
}

namespace {

// The canary word's line, after a block's usable bytes.
constexpr size_t kCanaryBytes = 128;

// Uncached / fine-grained blocks are never handed back to the runtime while
// the process lives: memory freed with hipFree after such an allocation was
// seen coming back from later plain hipMalloc calls with broken semantics
// (host-memory runs of the GPU suite gave wrong results in later, unrelated
// tests of the same process -- even one-rank runs that allocate no
// uncached memory at all -- and more of them the more uncached memory had
// been freed).  Freed ones wait here, per device and kind,
// for the next context to take them.
struct KindCache {
  std::mutex mu;
  struct Entry {
    int device;
    unsigned flags;
    size_t bytes;
    char* ptr;
  };
  std::vector<Entry> free;
};

KindCache& kindCache() {
  static KindCache* c = new KindCache();  // outlives every Context (never destroyed)
  return *c;
}

char* takeCached(int device, unsigned flags, size_t bytes, size_t* got, size_t cap) {
  KindCache& c = kindCache();
  std::lock_guard<std::mutex> g(c.mu);
  const size_t most = std::max(2 * bytes, bytes + (size_t(4) << 20));
  size_t best = c.free.size();
  for (size_t i = 0; i < c.free.size(); i++) {
    const auto& e = c.free[i];
    if (e.device == device && e.flags == flags && e.bytes >= bytes && e.bytes <= most &&
        e.bytes < cap && (best == c.free.size() || e.bytes < c.free[best].bytes)) {
      best = i;
    }
  }
  if (best == c.free.size()) return nullptr;
  char* p = c.free[best].ptr;
  *got = c.free[best].bytes;
  c.free.erase(c.free.begin() + (long)best);
  return p;
}

// Give a block of `flags` kind back: plain blocks to the runtime, the others
// to the cache above.
void freeBlock(int device, char* p, size_t bytes, unsigned flags) {
  if (p == nullptr) return;
  // GLOO_AMD_UC_CACHE=0 frees them like plain blocks (to reproduce the
  // hazard; never in production)
  static const bool cache = [] {
    const char* e = std::getenv("GLOO_AMD_UC_CACHE");
    return !(e != nullptr && e[0] == '0');
  }();
  if (flags == 0 || !cache) {
    GLX_TRACE_MEM("hipFree block %p (%zu, flags %u)", (void*)p, bytes, flags);
    hipFree(p);
    return;
  }
  GLX_TRACE_MEM("cache block %p (%zu, flags %u)", (void*)p, bytes, flags);
  KindCache& c = kindCache();
  std::lock_guard<std::mutex> g(c.mu);
  c.free.push_back(KindCache::Entry{device, flags, bytes, p});
}

// `bytes` in, the block's real size out (a cached block may be larger).
// cap: take no recycled block of cap bytes or more
char* allocBlock(int device, size_t* bytes, unsigned flags, size_t cap = SIZE_MAX) {
  char* d = nullptr;
  if (flags != 0) {
    size_t got = 0;
    d = takeCached(device, flags, *bytes, &got, cap);
    if (d != nullptr) {
      *bytes = got;
      return d;
    }
    GLX_HIP_CHECK(hipExtMallocWithFlags((void**)&d, *bytes, flags));
  } else {
    GLX_HIP_CHECK(hipMalloc((void**)&d, *bytes));
  }
  GLX_TRACE_MEM("alloc block %p (%zu, flags %u)", (void*)d, *bytes, flags);
  return d;
}
}  // namespace

Context::~Context() {
  if (shared_.empty() && imported_.empty()) return;
  if (device_ >= 0) hipSetDevice(device_);
  for (auto& kv : imported_) hipIpcCloseMemHandle(kv.second.opened);
  for (auto& b : shared_) freeBlock(device_, b.ptr, b.bytes + kCanaryBytes, b.flags);
}

namespace {

// Free pooled bytes kept beyond this are returned to the runtime.
constexpr size_t kMaxFreeSharedBytes = size_t(8) << 30;


// Allocation granule of a shared block: one 4 KiB page.  Round 1 rounded every block up to 2 MiB after a
// peer's mapping of a small block was seen pointing elsewhere; with every
// import now checked against the exporter's canary (and corrected by the
// published base offset if the runtime maps the allocation's base), 4 KiB
// blocks passed 8-rank runs with ~120 checked imports per rank, no fixup and
// no mismatch, so the granule is back to a page.
size_t sharedGranule() { return 4096; }

std::atomic<uint64_t> g_canary_counter{0};

uint64_t makeCanary(int rank, int64_t id) {
  // splitmix64 of (pid, rank, id, a process-wide counter, the clock)
  uint64_t x = ((uint64_t)::getpid() << 32) ^ ((uint64_t)rank << 20) ^ (uint64_t)id ^
               (g_canary_counter.fetch_add(1) << 44) ^
               (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x == 0 ? 1 : x;
}
}  // namespace

size_t Context::ipcMaxBlockBytes() {
  static const size_t v = [] {
    const char* e = std::getenv("GLOO_AMD_IPC_MAX_BLOCK_BYTES");
    const long long x = e != nullptr ? std::atoll(e) : 0;
    return x >= (1 << 20) ? (size_t)x : kIpcMaxBlockBytes;
  }();
  return v;
}

SharedBlock Context::acquireShared(size_t bytes, unsigned flags) {
  const size_t granule = sharedGranule();
  const size_t alloc =
      (std::max<size_t>(bytes, 1) + kCanaryBytes + granule - 1) / granule * granule;
  bytes = alloc - kCanaryBytes;
  // A peer process's hipIpcOpenMemHandle of an allocation of 2^31 bytes or
  // more never returns under the HIP runtime torch ships (ROCm 7.0; the
  // image's 7.2 runtime maps it: tools/micro/ipc_size_probe.py),
  // so such a block is refused here rather than hanging both ranks.
  GLX_ENFORCE(!sharesAcrossProcesses() || alloc < ipcMaxBlockBytes(), "rank ", rank,
              ": a landing block of ", alloc, " bytes would have to be shared with another "
              "process, and IPC imports of ", ipcMaxBlockBytes(), " bytes or more hang in "
              "the HIP runtime torch ships (GLOO_AMD_IPC_MAX_BLOCK_BYTES raises the limit "
              "for a runtime that maps more); this schedule's largest receive region needs "
              "it (use a smaller buffer per call, more ranks, or the ring / "
              "halving-doubling schedule, whose messages are split)");
  std::lock_guard<std::mutex> g(sharedMutex_);
  // the smallest free block of this kind that fits without wasting much
  SharedBlock* best = nullptr;
  const size_t most = std::max(2 * bytes, bytes + (size_t(4) << 20));
  for (auto& b : shared_) {
    if (!b.inUse && b.flags == flags && b.bytes >= bytes && b.bytes <= most &&
        (best == nullptr || b.bytes < best->bytes)) {
      best = &b;
    }
  }
  if (best != nullptr) {
    best->inUse = true;
    return *best;
  }
  SharedBlock nb;
  size_t got = alloc;
  // a recycled block may be larger (never as large as the IPC limit)
  nb.ptr = allocBlock(device_, &got, flags, ipcMaxBlockBytes());
  bytes = got - kCanaryBytes;
  nb.bytes = bytes;
  nb.flags = flags;
  nb.ref.ptr = (uint64_t)(uintptr_t)nb.ptr;
  nb.ref.id = nextSharedId_++;
  // exported only when some peer is another process: thread-ranks of this
  // process use the pointer itself, and an IPC export (a dmabuf the runtime
  // keeps per allocation) is one more thing the block's memory carries
  if (size > 1 && crossProcess_) {
    std::memset(&nb.ref.ipc, 0, sizeof(nb.ref.ipc));
    const hipError_t e = hipIpcGetMemHandle(&nb.ref.ipc, nb.ptr);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      freeBlock(device_, nb.ptr, got, flags);
      GLX_ENFORCE(false, "rank ", rank, ": hipIpcGetMemHandle of a ", got,
                  "-byte shared block refused: ", hipGetErrorName(e), " (", hipGetErrorString(e),
                  ")");
    }
    nb.ref.ipcStatus = 1;
    void* base = nullptr;
    size_t range = 0;
    if (hipMemGetAddressRange(&base, &range, nb.ptr) == hipSuccess && base != nullptr) {
      nb.ref.baseOff = (uint64_t)(nb.ptr - static_cast<char*>(base));
    } else {
      (void)hipGetLastError();
    }
    nb.ref.canaryOff = bytes;
    nb.ref.canary = makeCanary(rank, nb.ref.id);
    GLX_HIP_CHECK(hipMemcpy(nb.ptr + nb.ref.canaryOff, &nb.ref.canary, sizeof(uint64_t),
                            hipMemcpyHostToDevice));
  }
  nb.inUse = true;
  shared_.push_back(nb);
  return nb;
}

void Context::releaseShared(int64_t id) {
  std::lock_guard<std::mutex> g(sharedMutex_);
  size_t freeBytes = 0;
  for (auto& b : shared_) {
    if (b.ref.id == id) b.inUse = false;
    if (!b.inUse) freeBytes += b.bytes;
  }
  // over the cap: return the largest free blocks (the id is never reused;
  // peers close their mappings when they see it retired in our next
  // algorithm record)
  while (freeBytes > kMaxFreeSharedBytes) {
    auto big = shared_.end();
    for (auto it = shared_.begin(); it != shared_.end(); ++it) {
      if (!it->inUse && (big == shared_.end() || it->bytes > big->bytes)) big = it;
    }
    if (big == shared_.end()) break;
    freeBytes -= big->bytes;
    freeBlock(device_, big->ptr, big->bytes + kCanaryBytes, big->flags);
    retired_.push_back(big->ref.id);
    shared_.erase(big);
  }
}

std::vector<int64_t> Context::retiredShared() {
  std::lock_guard<std::mutex> g(sharedMutex_);
  return retired_;
}

void Context::dropImported(int r, const std::vector<int64_t>& ids) {
  std::lock_guard<std::mutex> g(sharedMutex_);
  for (int64_t id : ids) {
    auto it = imported_.find({r, id});
    if (it == imported_.end()) continue;
    hipIpcCloseMemHandle(it->second.opened);
    imported_.erase(it);
  }
}

char* Context::importShared(int r, const SharedRef& ref) {
  std::lock_guard<std::mutex> g(sharedMutex_);
  auto it = imported_.find({r, ref.id});
  if (it != imported_.end()) return it->second.ptr;
  GLX_ENFORCE(ref.ipcStatus == 1, "rank ", r, " published shared block ", ref.id,
              " without an IPC handle");
  void* p = nullptr;
  GLX_TRACE("r%d import: rank %d shared block %ld (%lu bytes)", rank, r, (long)ref.id,
            (unsigned long)ref.canaryOff);
  GLX_HIP_CHECK(hipIpcOpenMemHandle(&p, ref.ipc, hipIpcMemLazyEnablePeerAccess));
  GLX_TRACE("r%d import: opened at %p", rank, p);
  auto canaryAt = [&](const char* at) -> uint64_t {
    uint64_t v = 0;
    const hipError_t e = hipMemcpy(&v, at + ref.canaryOff, sizeof(v), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    return v;
  };
  char* at = static_cast<char*>(p);
  const uint64_t seen = canaryAt(at);
  ipcImports_++;
  if (seen != ref.canary) {
    // the runtime may hand back the base of the exporter's allocation
    // rather than the exported pointer inside it
    if (ref.baseOff != 0 && canaryAt(at + ref.baseOff) == ref.canary) {
      at += ref.baseOff;
      ipcBaseFixups_++;
    } else {
      hipIpcCloseMemHandle(p);
      GLX_ENFORCE(false, "rank ", rank, ": the IPC mapping of rank ", r, "'s shared block ",
                  ref.id, " does not hold its canary (read 0x", std::hex, seen, ", expected 0x",
                  ref.canary, std::dec, "; block at offset ", ref.baseOff,
                  " in its allocation): the mapping is not the exporter's memory");
    }
  }
  imported_[{r, ref.id}] = Imported{p, at};
  return at;
}

void Context::clearOps() {
  std::map<std::string, std::shared_ptr<Algorithm>> drop;
  {
    std::lock_guard<std::mutex> g(opsMutex);
    drop.swap(ops);
  }
  drop.clear();  // executors release their reference to this context here
}

int Context::nextSlot(int numToSkip) {
  GLX_ENFORCE(numToSkip > 0, "numToSkip must be > 0");
  int s = slot_;
  slot_ += numToSkip;
  return s;
}

void Context::connectFullMesh(std::shared_ptr<rendezvous::Store> store) {
  GLX_ENFORCE(!connected_, "context already connected");
  store_ = std::move(store);
  busId_ = busIdOf(device_);
  const pid_t pid = ::getpid();
  // Name unique on the node: pid + per-process counter + rank.
  const std::string shm = "/glx." + std::to_string(pid) + "." +
                          std::to_string(g_ctx_counter.fetch_add(1)) + ".r" +
                          std::to_string(rank);
  local_.create(shm);

  std::vector<char> rec;
  putPod<uint32_t>(rec, 0x474c5831u);  // "GLX1"
  putPod<int32_t>(rec, rank);
  putPod<int32_t>(rec, size);
  putPod<int64_t>(rec, (int64_t)pid);
  putPod<int32_t>(rec, device_);
  putStr(rec, busId_);
  putStr(rec, shm);
  putPod<int32_t>(rec, hwQueuesOfProcess());
  store_->set("glx/ep/" + std::to_string(rank), rec);

  for (int r = 0; r < size; r++) {
    PeerEndpoint& p = peers_[r];
    p.rank = r;
    if (r == rank) {
      p.pid = pid;
      p.device = device_;
      p.localDevice = device_;
      p.sameProcess = true;
      p.busId = busId_;
      p.shmName = shm;
      p.hwQueues = hwQueuesOfProcess();
      continue;
    }
    auto b = store_->get("glx/ep/" + std::to_string(r), timeout_);
    Reader rd{b};
    GLX_ENFORCE(rd.pod<uint32_t>() == 0x474c5831u, "bad endpoint record from rank ", r);
    GLX_ENFORCE(rd.pod<int32_t>() == r, "endpoint record rank mismatch");
    GLX_ENFORCE(rd.pod<int32_t>() == size, "peer ", r, " has a different context size");
    p.pid = (pid_t)rd.pod<int64_t>();
    p.device = rd.pod<int32_t>();
    std::string bus = rd.str();
    p.busId = bus;
    p.shmName = rd.str();
    p.hwQueues = rd.pod<int32_t>();
    p.sameProcess = (p.pid == pid);
    if (p.sameProcess) {
      p.localDevice = p.device;
    } else {
      int d = -1;
      if (!bus.empty() && hipDeviceGetByPCIBusId(&d, bus.c_str()) == hipSuccess) {
        p.localDevice = d;
      }
    }
    p.ctl.reset(new ControlBlock());
    p.ctl->open(p.shmName);
    if (p.localDevice >= 0 && p.localDevice != device_) {
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, device_, p.localDevice) != hipSuccess) {
        (void)hipGetLastError();
        can = 0;
      }
      p.canAccessPeer = can;
      if (can) {
        int cur = 0;
        hipGetDevice(&cur);
        hipSetDevice(device_);
        hipError_t e = hipDeviceEnablePeerAccess(p.localDevice, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
          hipSetDevice(cur);
          GLX_HIP_CHECK(e);
        }
        (void)hipGetLastError();  // clear "already enabled"
        hipSetDevice(cur);
      }
      int atomics = 0;
      if (hipDeviceGetP2PAttribute(&atomics, hipDevP2PAttrNativeAtomicSupported, device_,
                                   p.localDevice) != hipSuccess) {
        (void)hipGetLastError();
        atomics = 0;
      }
      p.nativeAtomics = atomics;
      if (atomics == 0) flagStores_ = true;
    }
  }
  if (const char* e = std::getenv("GLOO_AMD_FLAG_WRITE")) {
    if (std::strcmp(e, "store") == 0) flagStores_ = true;
    if (std::strcmp(e, "atomic") == 0) flagStores_ = false;
  }
  // Everyone has mapped everyone: the names can go (mappings stay valid and
  // nothing is left behind in /dev/shm if a rank dies later).
  store_->set("glx/ep/" + std::to_string(rank) + "/mapped", std::vector<char>(1, 1));
  for (int r = 0; r < size; r++) {
    if (r != rank) store_->get("glx/ep/" + std::to_string(r) + "/mapped", timeout_);
  }
  local_.unlink();
  crossProcess_ = false;
  for (const auto& p : peers_) crossProcess_ = crossProcess_ || !p.sameProcess;
  connected_ = true;
}

bool Context::ranksShareDevice() const {
  for (size_t a = 0; a < peers_.size(); a++) {
    for (size_t b = a + 1; b < peers_.size(); b++) {
      if (peers_[a].pid == peers_[b].pid && peers_[a].device == peers_[b].device) return true;
    }
  }
  return false;
}

// Hardware queues this process opens per device (HIP's GPU_MAX_HW_QUEUES,
// default 4).  Published in the endpoint record, so every rank decides on
// the device engines from the same (largest) value.
int hwQueuesOfProcess() {
  const char* e = std::getenv("GPU_MAX_HW_QUEUES");
  const int n = e != nullptr ? std::atoi(e) : 0;
  return n > 0 ? n : 4;
}

int Context::maxHwQueues() const {
  int most = 1;
  for (const auto& p : peers_) most = std::max(most, p.hwQueues);
  return most;
}

int Context::maxRanksPerDevice() const {
  std::map<std::string, int> n;
  int most = 1;
  for (const auto& p : peers_) {
    const std::string key = !p.busId.empty()
                                ? p.busId
                                : std::to_string(p.pid) + ":" + std::to_string(p.device);
    most = std::max(most, ++n[key]);
  }
  return most;
}

namespace {
// A killed process stays a zombie until its parent reaps it; kill(pid, 0)
// still succeeds then, /proc/<pid>/stat says 'Z' (or 'X').
bool processGone(pid_t pid) {
  if (::kill(pid, 0) != 0) return errno == ESRCH;
  char path[64];
  std::snprintf(path, sizeof(path), "/proc/%d/stat", (int)pid);
  FILE* f = std::fopen(path, "r");
  if (f == nullptr) return false;
  char buf[512];
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* rp = std::strrchr(buf, ')');  // comm may hold spaces and ')'
  return rp != nullptr && rp[1] == ' ' && (rp[2] == 'Z' || rp[2] == 'X');
}
}  // namespace

int Context::deadPeer() const {
  for (const auto& p : peers_) {
    if (p.rank == rank || p.sameProcess || p.pid <= 0) continue;
    if (processGone(p.pid)) return p.rank;
  }
  return -1;
}

void Context::checkPeersAlive() {
  const int r = deadPeer();
  if (r >= 0) {
    GLX_THROW_IO("Connection closed by peer: rank ", r, " (pid ", peers_[(size_t)r].pid,
                 ") exited");
  }
}

}  // namespace gloo
