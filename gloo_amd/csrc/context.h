// context.h -- gloo::Context for the in-node xGMI device transport.
//
// Replaces gloo::Context (gloo/context.h:26-58) + rendezvous::Context
// (gloo/rendezvous/context.h:25-35) + the transport Device/Pair factory
// (gloo/transport/device.h:49, gloo/transport/pair.h:33-37).
//
// Data never touches the host: payload moves GPU->GPU with
// hipMemcpyPeerAsync into the peer's device receive regions.  What the TCP
// transport does with sockets and an epoll thread (completion of a message,
// "inbox free" notifications) is done here with 64-bit monotonic counters in
// a per-rank POSIX shared-memory control block that every rank of the node
// maps: a sender bumps the receiver's delivery counter once its copy has
// completed (observed with hipEventQuery), a receiver bumps the sender's
// credit counter once the kernel that consumed the message has completed.
// Ranks may be threads of one process (the reference's test topology,
// gloo/test/base_test.h:91-166) or one process per GPU (torchrun).
#pragma once

#include <hip/hip_runtime_api.h>
#include <sys/types.h>

#include <atomic>
#include <chrono>
#include <map>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "store.h"

namespace gloo {

class Algorithm;

// One rank's control block: kWords counters, one per 64-byte line.
class ControlBlock {
 public:
  static constexpr size_t kWords = 16384;
  static constexpr size_t kLine = 64;
  static constexpr size_t kBytes = kWords * kLine;

  ControlBlock() = default;
  ~ControlBlock();
  ControlBlock(const ControlBlock&) = delete;
  ControlBlock& operator=(const ControlBlock&) = delete;

  void create(const std::string& name);  // shm_open(O_CREAT) + mmap
  void open(const std::string& name);    // map a peer's block
  void unlink();                         // drop the name (mappings stay)

  std::atomic<uint64_t>* word(uint32_t i) const {
    return reinterpret_cast<std::atomic<uint64_t>*>(base_ + (size_t)i * kLine);
  }
  const std::string& name() const { return name_; }

  // Local word allocator (only on the owner's block).
  uint32_t allocWord();
  void freeWord(uint32_t i);

 private:
  std::string name_;
  char* base_ = nullptr;
  bool owner_ = false;
  bool unlinked_ = false;
  std::mutex m_;
  std::vector<uint32_t> free_;
  uint32_t next_ = 1;  // word 0 reserved
};

struct PeerEndpoint {
  int rank = -1;
  pid_t pid = 0;
  int device = -1;       // device ordinal in the peer's process
  int localDevice = -1;  // the same GPU's ordinal in this process (-1: unknown)
  bool sameProcess = false;
  std::string busId;  // PCI bus id of the rank's GPU ("" if unknown)
  // read at connect when the peer's GPU is another one of this process's
  // devices (-1 otherwise): hipDeviceCanAccessPeer, and
  // hipDevP2PAttrNativeAtomicSupported of the link (0 -> flag stores)
  int canAccessPeer = -1;
  int nativeAtomics = -1;
  std::string shmName;
  int hwQueues = 4;  // the rank's process's GPU_MAX_HW_QUEUES (default 4)
  std::unique_ptr<ControlBlock> ctl;  // mapped peer control block
};

int hwQueuesOfProcess();

// What a peer needs to map one of our shared device blocks (published in
// algorithm records).
struct SharedRef {
  uint64_t ptr = 0;         // our address (threads of our process use it as is)
  int64_t id = 0;           // unique within the exporting context, never reused
  int32_t ipcStatus = 0;    // 1 exported (always, when the context has peers)
  hipIpcMemHandle_t ipc{};  // hipIpcGetMemHandle(ptr)
  uint64_t canaryOff = 0;   // the canary word sits at ptr + canaryOff
  uint64_t canary = 0;      // its value, written by the exporter at allocation
  uint64_t baseOff = 0;     // ptr - base of the runtime allocation holding it
                            // (hipMemGetAddressRange)
};

// Device memory peers map (receive regions, landing slots, flag rows).
struct SharedBlock {
  char* ptr = nullptr;
  size_t bytes = 0;     // usable bytes (the canary lies beyond them)
  unsigned flags = 0;   // 0: hipMalloc, else hipExtMallocWithFlags
  SharedRef ref;
  bool inUse = false;
};

class Context {
 public:
  Context(int rank, int size, int device);
  ~Context();

  const int rank;
  const int size;

  int device() const { return device_; }
  // gloo::Context::base (gloo/context.h:33): ranks per group of the class
  // AllreduceBcube created afterwards (default 2)
  int base() const { return base_; }
  void setBase(int b) { base_ = b; }

  // gloo/rendezvous/context.cc:43-113
  void connectFullMesh(std::shared_ptr<rendezvous::Store> store);
  bool connected() const { return connected_; }

  int nextSlot(int numToSkip = 1);  // gloo/context.cc:49-54

  void setTimeout(std::chrono::milliseconds t) { timeout_ = t; }  // gloo/context.cc:61
  std::chrono::milliseconds getTimeout() const { return timeout_; }

  rendezvous::Store& store() { return *store_; }
  ControlBlock& localControl() { return local_; }
  PeerEndpoint& peer(int r) { return peers_.at(r); }

  // True when two ranks of the context are threads of one process on one
  // device (the same answer on every rank: it is computed from all
  // endpoints).  Their streams may share a hardware queue, so kernels that
  // wait for each other on the device could not both run.
  bool ranksShareDevice() const;
  // Largest number of ranks on one GPU (by PCI bus id; equal on every rank).
  int maxRanksPerDevice() const;
  // the largest GPU_MAX_HW_QUEUES of any rank's process (from the endpoints)
  int maxHwQueues() const;
  // True when device kernels of this rank write peers' flag words with plain
  // system-scope stores instead of atomic exchanges: some peer sits on
  // another GPU whose link (hipDevP2PAttrNativeAtomicSupported) does not
  // carry atomics, or GLOO_AMD_FLAG_WRITE=store.
  bool flagStores() const { return flagStores_; }

  // Throws IoException if a peer process has exited.
  void checkPeersAlive();
  // rank of a peer process that has exited, or -1
  int deadPeer() const;

  // Shared device blocks, pooled per context: an algorithm takes a block
  // (allocated and IPC-exported once, or a free one of a fitting size) and
  // gives it back when it is destroyed; a peer's block is imported once
  // (by rank and block id) and stays mapped until the context goes.  Creating
  // and destroying algorithms then costs no IPC export / import / close
  // after the first few -- those calls are slow and, with many processes
  // exporting at once, were seen to fail.
  //
  // Every exported block carries a canary word beyond its usable bytes; an
  // importer checks it before using the mapping and throws EnforceNotMet if
  // the mapping does not hold it (a mapping of some other memory would
  // otherwise corrupt data or lose flags silently).
  //
  // A block another process imports stays below kIpcMaxBlockBytes (with its
  // canary and page rounding): larger ones are refused with EnforceNotMet,
  // since a peer's hipIpcOpenMemHandle of 2^31 bytes or more never returned
  // under torch's HIP runtime (2^31 - 2 MiB mapped).
  // GLOO_AMD_IPC_MAX_BLOCK_BYTES raises it for a runtime that maps more (the
  // image's ROCm 7.2 runtime maps 4 GiB); every rank must use the
  // same value.  Messages above 512 MiB are split (plan.h kMaxMessageBytes),
  // so the default limit is reached only by an explicit schedule's own slot
  // arrays (the one-shot's whole buffers) or glx_set_max_message_bytes.
  static constexpr size_t kIpcMaxBlockBytes = size_t(1) << 31;
  static size_t ipcMaxBlockBytes();
  bool sharesAcrossProcesses() const { return size > 1 && crossProcess_; }
  SharedBlock acquireShared(size_t bytes, unsigned flags);
  void releaseShared(int64_t id);
  char* importShared(int rank, const SharedRef& ref);
  // Blocks this context returned to the runtime (over the pool's cap), by
  // id: published in every algorithm record so that peers close their
  // mappings of them (the physical memory is freed only when every importer
  // has closed its handle).
  std::vector<int64_t> retiredShared();
  // Close our imports of rank r's blocks `ids` (those it has retired).
  void dropImported(int r, const std::vector<int64_t>& ids);
  // Imports whose mapping the runtime returned at the base of the exporter's
  // allocation instead of at the exported pointer (the canary was found at
  // baseOff further on), and imports checked in all.
  int64_t ipcBaseFixups() const { return ipcBaseFixups_; }
  int64_t ipcImports() const { return ipcImports_; }

  // Executors of function-style collectives by options key (see
  // collectives.cc).  They hold a reference to this context: clearOps()
  // breaks that cycle when the context's owner lets go of it.
  std::mutex opsMutex;
  std::map<std::string, std::shared_ptr<Algorithm>> ops;
  void clearOps();

 private:
  int device_;
  int base_ = 2;
  int slot_ = 0;
  bool connected_ = false;
  bool flagStores_ = false;
  bool crossProcess_ = true;  // some peer is another process (set at connect)
  std::chrono::milliseconds timeout_{30000};  // gloo/context.cc:18
  std::shared_ptr<rendezvous::Store> store_;
  ControlBlock local_;
  std::vector<PeerEndpoint> peers_;
  std::string busId_;
  std::mutex sharedMutex_;
  std::vector<SharedBlock> shared_;
  int64_t nextSharedId_ = 1;
  struct Imported {
    void* opened;  // what hipIpcOpenMemHandle returned (closed at the end)
    char* ptr;     // the exporter's block
  };
  std::map<std::pair<int, int64_t>, Imported> imported_;
  int64_t ipcBaseFixups_ = 0, ipcImports_ = 0;
  std::vector<int64_t> retired_;
};

}  // namespace gloo
