// host_fn.cc -- the function-style allreduce with a caller's reduction
// function, on host buffers (host_fn.h).
#include "host_fn.h"

#include <fcntl.h>
#include <immintrin.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <thread>

#include "common.h"

namespace gloo {

namespace {

constexpr uint32_t kHostFnMagic = 0x67686678;  // record of one rank's host-fn executor
constexpr int32_t kDirIn = 0, kDirOut = 1;
std::atomic<uint64_t> g_regionSerial{0};

template <typename T>
void put(std::vector<char>& b, T v) {
  const char* p = reinterpret_cast<const char*>(&v);
  b.insert(b.end(), p, p + sizeof(T));
}

template <typename T>
T take(const std::vector<char>& b, size_t& at) {
  GLX_ENFORCE(at + sizeof(T) <= b.size(), "host-fn allreduce: truncated peer record");
  T v;
  std::memcpy(&v, b.data() + at, sizeof(T));
  at += sizeof(T);
  return v;
}

char* mapShm(const std::string& name, size_t bytes, bool create) {
  const int fd = create ? ::shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600)
                        : ::shm_open(name.c_str(), O_RDWR, 0600);
  if (fd < 0) GLX_THROW_IO("shm_open(", name, ") failed: ", std::strerror(errno));
  if (create && ::ftruncate(fd, (off_t)bytes) != 0) {
    const int e = errno;
    ::close(fd);
    ::shm_unlink(name.c_str());
    GLX_THROW_IO("ftruncate(", name, ", ", bytes, ") failed: ", std::strerror(e));
  }
  void* p = ::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) GLX_THROW_IO("mmap(", name, ") failed: ", std::strerror(errno));
  return static_cast<char*>(p);
}

}  // namespace

HostFnExecutor::HostFnExecutor(const std::shared_ptr<Context>& ctx, int algo,
                               size_t elementSize, size_t elements, size_t maxSegmentBytes)
    : Algorithm(ctx), algo_(algo), es_(elementSize), elements_(elements) {
  const bool cls = algo == glx::ALGO_RING_CHUNKED || algo == glx::ALGO_HALVING_DOUBLING;
  GLX_ENFORCE(algo == glx::ALGO_FN_RING || algo == glx::ALGO_FN_BCUBE || cls,
              "host-fn allreduce: RING or BCUBE, or the class ring_chunked / "
              "halving_doubling");
  GLX_ENFORCE(es_ > 0 && es_ <= (size_t(1) << 20), "host-fn allreduce: bad element size ", es_);
  glx::PlanParams prm;
  prm.esize = (int)es_;
  prm.maxSegmentBytes = (int64_t)maxSegmentBytes;
  prm.minPieceBytes = 0;  // the reference's own segments (nothing to pipeline on the host)
  plan_ = glx::makePlan(algo, contextRank_, contextSize_, (int64_t)elements, prm);
  for (const auto& s : plan_.steps) {
    GLX_ENFORCE(s.kind != glx::FOLD || (s.flags & glx::kFoldWhole) == 0,
                "host-fn allreduce: whole-buffer folds are not expected here");
    // a class algorithm's function is x = f(x, y) (host_fn.h): its programs
    // reduce in place only
    GLX_ENFORCE(!cls || s.kind != glx::FOLD, "host-fn allreduce: a class program folds");
  }
  slot_ = ctx->nextSlot();
  regionBytes_ = std::max<size_t>(64, (size_t)plan_.scratch_elems * es_ + 64);
  if (contextSize_ > 1 && elements > 0) {
    // this rank's landing regions: shared memory its peers map
    shmName_ = "/glx_hfn_" + std::to_string(::getpid()) + "_" + std::to_string(contextRank_) +
               "_" + std::to_string(g_regionSerial.fetch_add(1));
    region_ = mapShm(shmName_, regionBytes_, true);
    auto& ctl = ctx->localControl();
    stepChan_.assign(plan_.steps.size(), -1);
    for (size_t i = 0; i < plan_.steps.size(); i++) {
      const auto& s = plan_.steps[i];
      if (s.kind == glx::SEND) {
        stepChan_[i] = chanIndex(out_, (int)s.peer, s.channel);
      } else if (s.kind == glx::RECV || s.kind == glx::RELEASE) {
        stepChan_[i] = chanIndex(in_, (int)s.peer, s.channel);
      }
    }
    for (auto& c : out_) c.word = ctl.allocWord();  // our credit words
    for (auto& c : in_) c.word = ctl.allocWord();   // our delivery words
    publish();
  }
}

HostFnExecutor::~HostFnExecutor() noexcept(false) {
  auto& ctl = context_->localControl();
  // every receiver's credit for our last message before our credit words go
  // back to the control block: a credit landing late in a word a later
  // algorithm was given would corrupt that algorithm's counts (a class
  // algorithm can be freed and another created on the same context)
  if (!broken_) {
    const auto deadline = std::chrono::steady_clock::now() + context_->getTimeout();
    try {
      for (auto& c : out_) {
        std::atomic<uint64_t>* credit = ctl.word(c.word);
        while (credit->load(std::memory_order_acquire) < c.count &&
               std::chrono::steady_clock::now() < deadline) {
          context_->checkPeersAlive();  // throws if a peer exited: stop waiting
          std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
      }
    } catch (...) {
    }
  }
  for (auto& c : out_) ctl.freeWord(c.word);
  for (auto& c : in_) ctl.freeWord(c.word);
  for (size_t r = 0; r < peerRegion_.size(); r++) {
    if (peerRegion_[r] != nullptr) ::munmap(peerRegion_[r], peerBytes_[r]);
  }
  if (region_ != nullptr) ::munmap(region_, regionBytes_);
  if (!shmName_.empty() && !unlinked_) ::shm_unlink(shmName_.c_str());
}

void HostFnExecutor::run() {
  GLX_ENFORCE(false, "host-fn allreduce: call through gloo::allreduce(opts)");
}

int HostFnExecutor::chanIndex(std::vector<Chan>& v, int peer, int64_t tag) {
  for (size_t i = 0; i < v.size(); i++) {
    if (v[i].peer == peer && v[i].tag == tag) return (int)i;
  }
  Chan c;
  c.peer = peer;
  c.tag = tag;
  v.push_back(c);
  return (int)v.size() - 1;
}

// Where our messages land (the shared-memory name and size) and which of our
// counter words the peers bump (delivery) or watch (credit).
void HostFnExecutor::publish() {
  std::vector<char> b;
  put<uint32_t>(b, kHostFnMagic);
  put<int32_t>(b, (int32_t)algo_);
  put<uint64_t>(b, (uint64_t)es_);
  put<uint64_t>(b, (uint64_t)elements_);
  put<uint64_t>(b, (uint64_t)regionBytes_);
  put<uint32_t>(b, (uint32_t)shmName_.size());
  b.insert(b.end(), shmName_.begin(), shmName_.end());
  put<uint32_t>(b, (uint32_t)(in_.size() + out_.size()));
  for (const auto& c : in_) {
    put<int32_t>(b, c.peer);
    put<int64_t>(b, c.tag);
    put<int32_t>(b, kDirIn);
    put<uint32_t>(b, c.word);
  }
  for (const auto& c : out_) {
    put<int32_t>(b, c.peer);
    put<int64_t>(b, c.tag);
    put<int32_t>(b, kDirOut);
    put<uint32_t>(b, c.word);
  }
  context_->store().set(
      "glx/hostfn/" + std::to_string(slot_) + "/" + std::to_string(contextRank_), b);
}

void HostFnExecutor::resolve() {
  peerRegion_.assign((size_t)contextSize_, nullptr);
  peerBytes_.assign((size_t)contextSize_, 0);
  std::vector<int> peers;
  for (const auto& c : out_) peers.push_back(c.peer);
  for (const auto& c : in_) peers.push_back(c.peer);
  std::sort(peers.begin(), peers.end());
  peers.erase(std::unique(peers.begin(), peers.end()), peers.end());
  for (int r : peers) {
    const auto rec = context_->store().get(
        "glx/hostfn/" + std::to_string(slot_) + "/" + std::to_string(r),
        context_->getTimeout());
    size_t at = 0;
    GLX_ENFORCE(take<uint32_t>(rec, at) == kHostFnMagic, "host-fn allreduce: bad record of rank ",
                r);
    const int32_t algo = take<int32_t>(rec, at);
    const uint64_t es = take<uint64_t>(rec, at), n = take<uint64_t>(rec, at);
    GLX_ENFORCE(algo == algo_ && es == es_ && n == elements_, "rank ", r,
                "'s allreduce in slot ", slot_, " (algorithm ", algo, ", element size ", es,
                ", elements ", n, ") differs from rank ", contextRank_, "'s (", algo_, ", ", es_,
                ", ", elements_, "): the ranks called allreduce differently");
    const uint64_t bytes = take<uint64_t>(rec, at);
    const uint32_t len = take<uint32_t>(rec, at);
    GLX_ENFORCE(at + len <= rec.size(), "host-fn allreduce: truncated peer record");
    const std::string name(rec.data() + at, len);
    at += len;
    bool sendsTo = false;
    for (const auto& c : out_) sendsTo = sendsTo || c.peer == r;
    if (sendsTo) {
      peerRegion_[(size_t)r] = mapShm(name, (size_t)bytes, false);
      peerBytes_[(size_t)r] = (size_t)bytes;
    }
    PeerEndpoint& pe = context_->peer(r);
    GLX_ENFORCE(pe.ctl != nullptr, "host-fn allreduce: no control block of rank ", r);
    const uint32_t nchan = take<uint32_t>(rec, at);
    for (uint32_t k = 0; k < nchan; k++) {
      const int32_t peer = take<int32_t>(rec, at);
      const int64_t tag = take<int64_t>(rec, at);
      const int32_t dir = take<int32_t>(rec, at);
      const uint32_t word = take<uint32_t>(rec, at);
      if (peer != contextRank_) continue;
      if (dir == kDirIn) {  // r receives from us on `tag`: its delivery word
        for (auto& c : out_) {
          if (c.peer == r && c.tag == tag) c.peerWord = pe.ctl->word(word);
        }
      } else {  // r sends to us on `tag`: its credit word
        for (auto& c : in_) {
          if (c.peer == r && c.tag == tag) c.peerWord = pe.ctl->word(word);
        }
      }
    }
  }
  for (const auto& c : out_) {
    GLX_ENFORCE(c.peerWord != nullptr, "rank ", c.peer, " has no receive channel ", c.tag,
                " from rank ", contextRank_, " (schedules disagree)");
  }
  for (const auto& c : in_) {
    GLX_ENFORCE(c.peerWord != nullptr, "rank ", c.peer, " has no send channel ", c.tag,
                " to rank ", contextRank_, " (schedules disagree)");
  }
  resolved_ = true;
}

template <typename Pred>
void HostFnExecutor::waitFor(Pred done, const char* what, int peer,
                             std::chrono::milliseconds timeout) {
  if (done()) return;
  const auto start = std::chrono::steady_clock::now();
  auto lastAlive = start;
  for (uint64_t spin = 1;; spin++) {
    if (done()) return;
    if ((spin & 255) == 0) {
      const auto now = std::chrono::steady_clock::now();
      if (now - start > timeout) {
        GLX_THROW_TIMEOUT("Timed out waiting for ", what, " from rank ", peer, " (rank ",
                          contextRank_, ", host-fn allreduce, timeout ", timeout.count(),
                          " ms)");
      }
      if (now - lastAlive > std::chrono::milliseconds(200)) {
        lastAlive = now;
        context_->checkPeersAlive();  // throws IoException naming an exited peer
      }
    }
    if (spin > 4096) {
      std::this_thread::yield();
    } else {
      _mm_pause();
    }
  }
}

void HostFnExecutor::call(HostReduceFn fn, void* user, const std::vector<const void*>& in,
                          const std::vector<void*>& out, std::chrono::milliseconds timeout) {
  GLX_ENFORCE(fn != nullptr, "host-fn allreduce: null reduction function");
  GLX_ENFORCE(!out.empty(), "host-fn allreduce: at least one output is required");
  if (elements_ == 0) return;
  // every call of the caller's function; a failure stops this rank's call
  // here (its peers then time out waiting, as in the reference)
  auto f = [&](void* c, const void* a, const void* b, size_t n) {
    if (fn(user, c, a, b, n) != 0) {
      broken_ = true;
      throw std::invalid_argument("allreduce: the reduction function failed");
    }
  };
  const size_t bytes = elements_ * es_;
  char* out0 = static_cast<char*>(out[0]);
  // local reduction of the inputs into out[0] (gloo/allreduce.cc:44-82),
  // over the whole buffer: each element's happens once, before it is first
  // sent or reduced into, in the same operand order
  if (in.size() == 1) {
    if (in[0] != out0) std::memcpy(out0, in[0], bytes);
  } else if (in.size() >= 2) {
    f(out0, in[0], in[1], elements_);
    for (size_t i = 2; i < in.size(); i++) f(out0, out0, in[i], elements_);
  } else {
    for (size_t i = 1; i < out.size(); i++) f(out0, out0, out[i], elements_);
  }
  if (contextSize_ > 1) {
    const auto wait = timeout.count() > 0 ? timeout : context_->getTimeout();
    // a call that fails part-way leaves counts the peers never match: the
    // destructor then does not wait for credits
    broken_ = true;
    if (!resolved_) resolve();
    for (size_t i = 0; i < plan_.steps.size(); i++) {
      const glx::Step& s = plan_.steps[i];
      char* dst = out0 + (size_t)s.off * es_;
      const size_t len = (size_t)s.len * es_;
      switch (s.kind) {
        case glx::SEND: {
          Chan& c = out_[(size_t)stepChan_[i]];
          const uint64_t n = ++c.count;
          // one region per channel: message n lands once n - 1 was consumed
          std::atomic<uint64_t>* credit = context_->localControl().word(c.word);
          waitFor([&] { return credit->load(std::memory_order_acquire) + 1 >= n; },
                  "receive-region credit", c.peer, wait);
          if (len > 0) {
            std::memcpy(peerRegion_[(size_t)c.peer] + (size_t)s.dst_off * es_, dst, len);
          }
          c.peerWord->store(n, std::memory_order_release);
          break;
        }
        case glx::RECV: {
          Chan& c = in_[(size_t)stepChan_[i]];
          const uint64_t n = ++c.count;
          std::atomic<uint64_t>* delivery = context_->localControl().word(c.word);
          waitFor([&] { return delivery->load(std::memory_order_acquire) >= n; }, "data",
                  c.peer, wait);
          break;
        }
        case glx::REDUCE:  // out = f(out, tmp) (:292-296, :586-592)
          f(dst, dst, region_ + (size_t)s.boff * es_, (size_t)s.len);
          break;
        case glx::COPY:
          std::memcpy(dst, region_ + (size_t)s.boff * es_, len);
          break;
        case glx::FOLD: {  // bcube: out = f(out, peer) for the group's peers in order
          const auto& srcs = plan_.folds[(size_t)s.boff];
          auto src = [&](int64_t r) -> const void* {
            return r < 0 ? static_cast<const void*>(dst) : region_ + (size_t)r * es_;
          };
          if (!srcs.empty() && srcs[0] >= 0) std::memcpy(dst, src(srcs[0]), len);
          const bool left = (s.flags & glx::kFoldLeft) != 0;
          for (size_t k = 1; k < srcs.size(); k++) {
            if (left) {
              f(dst, dst, src(srcs[k]), (size_t)s.len);
            } else {
              f(dst, src(srcs[k]), dst, (size_t)s.len);
            }
          }
          break;
        }
        case glx::RELEASE: {
          Chan& c = in_[(size_t)stepChan_[i]];
          c.peerWord->store(++c.consumed, std::memory_order_release);
          break;
        }
        default:
          GLX_ENFORCE(false, "bad plan step kind ", s.kind);
      }
    }
    // every rank that sends to us has mapped our region by now (it resolved
    // before its first message, which this call received): drop the name
    if (!unlinked_ && !shmName_.empty()) {
      ::shm_unlink(shmName_.c_str());
      unlinked_ = true;
    }
    broken_ = false;
  }
  for (size_t i = 1; i < out.size(); i++) std::memcpy(out[i], out0, bytes);  // :87-96
  calls_++;
}

}  // namespace gloo
