// context.cc -- see context.h.
#include "context.h"

#include <algorithm>

#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstring>

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

Context::~Context() = default;

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
      if (hipDeviceCanAccessPeer(&can, device_, p.localDevice) == hipSuccess && can) {
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
    }
  }
  // Everyone has mapped everyone: the names can go (mappings stay valid and
  // nothing is left behind in /dev/shm if a rank dies later).
  store_->set("glx/ep/" + std::to_string(rank) + "/mapped", std::vector<char>(1, 1));
  for (int r = 0; r < size; r++) {
    if (r != rank) store_->get("glx/ep/" + std::to_string(r) + "/mapped", timeout_);
  }
  local_.unlink();
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

void Context::checkPeersAlive() {
  for (const auto& p : peers_) {
    if (p.rank == rank || p.sameProcess || p.pid <= 0) continue;
    if (::kill(p.pid, 0) != 0 && errno == ESRCH) {
      GLX_THROW_IO("Connection closed by peer: rank ", p.rank, " (pid ", p.pid,
                   ") exited");
    }
  }
}

}  // namespace gloo
