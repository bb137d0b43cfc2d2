// plan.cc -- compile the reference schedules into per-rank step programs.
//
// The element ranges, peers and orders of operations are those of the
// reference algorithms (cited per block); only the buffer management is
// ours: every incoming channel gets its own padded receive region in the
// rank's device scratch, and flow control is per-channel credits instead of
// the reference's separate notification buffers.
#include "plan.h"

#include <algorithm>
#include <cmath>
#include <atomic>
#include <map>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace glx {

namespace {

void fail(const std::string& what) { throw std::logic_error("plan: " + what); }

}  // namespace

// ---------------------------------------------------------------------------
// allreduce_ring_chunked (gloo/allreduce_ring_chunked.h)
// ---------------------------------------------------------------------------
Plan planRingChunked(int rank, int size, int64_t count) {
  Plan p;
  if (count == 0 || size == 1) return p;  // :47-49, :84-99
  const int64_t chunks = 2 * (int64_t)size;                       // :34
  const int64_t chunkSize = std::max<int64_t>(256, (count + chunks - 1) / chunks);  // :33,38
  const int64_t region = chunkSize + kPadElems;
  p.scratch_elems = 2 * region;  // inbox_[0], inbox_[1] (:43-45, sized to one chunk)
  const int left = (rank + size - 1) % size;
  const int right = (rank + 1) % size;

  auto chunk = [&](int64_t c, int64_t* off, int64_t* len) {  // :128-138
    int64_t o = c * chunkSize, l = chunkSize;
    if (o + l <= count) {
    } else if (o < count) {
      l = count - o;
    } else {
      l = 0;
    }
    *off = o;
    *len = l;
  };
  auto chunkOffset = [&](int round) -> int64_t {  // :125-127
    return ((2 * (int64_t)rank) - (round & ~1) + (round & 1) + chunks) % chunks;
  };
  auto send = [&](int64_t c) {  // copyChunkAtOffset, :215-236
    int64_t off, len;
    chunk(c % chunks, &off, &len);
    if (len == 0) off = 0;  // the reference's 1-element dummy becomes a bare signal
    p.steps.push_back({SEND, right, c & 1, off, len, 0, (c & 1) * region, 0});
    p.bytes_sent += len;
  };

  send(2 * (int64_t)rank);  // :102-103
  send(2 * (int64_t)rank + 1);
  for (int round = 2; round < chunks; round++) {  // reduce pass, :106-158
    const int64_t c = chunkOffset(round);
    int64_t off, len;
    chunk(c, &off, &len);
    p.steps.push_back({RECV, left, c & 1, 0, len, (c & 1) * region, 0, 0});
    if (len > 0) p.steps.push_back({REDUCE, 0, 0, off, len, (c & 1) * region, 0, 0});
    p.steps.push_back({RELEASE, left, c & 1, 0, 0, 0, 0, 0});
    send(c);
  }
  for (int round = 0; round < chunks - 2; round++) {  // broadcast pass, :163-200
    const int64_t c = chunkOffset(round);
    int64_t off, len;
    chunk(c, &off, &len);
    p.steps.push_back({RECV, left, c & 1, 0, len, (c & 1) * region, 0, 0});
    if (len > 0) p.steps.push_back({COPY, 0, 0, off, len, (c & 1) * region, 0, 0});
    p.steps.push_back({RELEASE, left, c & 1, 0, 0, 0, 0, 0});
    if (round < chunks - 4) send(c);
  }
  return p;
}

// ---------------------------------------------------------------------------
// allreduce_halving_doubling (gloo/allreduce_halving_doubling.h)
// ---------------------------------------------------------------------------
namespace {

uint32_t ilog2(uint32_t v) {
  uint32_t l = 0;
  while (v >>= 1) l++;
  return l;
}

uint32_t reverseBits(uint32_t v, uint32_t n) {  // :23-34
  uint32_t out = 0;
  for (uint32_t i = 0; i < n; i++) out |= ((v >> i) & 1u) << (n - 1 - i);
  return out;
}

struct HdGeom {
  int P = 0, rank = 0;
  int64_t count = 0, steps = 0, chunkSize = 0;
  // binary blocks (:39-64)
  uint32_t blockOff = 0, blockSize = 0, S = 0, rankInBlock = 0;
  uint32_t smaller = 0, larger = 0;
  std::vector<int64_t> sendOff, recvOff, sendCnt, recvCnt, stepChunk;
  int64_t stepChunkAfter = 0;
  int smallerPeer = -1;
  std::vector<int> largerPeers;
  int64_t sendCountToLarger = 0, totalToSend = 0;
  // receive regions of this rank
  std::vector<int64_t> regionStep;  // per step i
  int64_t regionSmaller = 0;
  std::vector<int64_t> regionLarger;  // per larger peer k
  int64_t scratch = 0;

  HdGeom(int P_, int rank_, int64_t count_) : P(P_), rank(rank_), count(count_) {
    steps = ilog2((uint32_t)P);                              // :76
    const int64_t chunks = (int64_t)1 << steps;              // :77
    chunkSize = (count + chunks - 1) / chunks;               // :78
    {
      uint32_t offset = (uint32_t)P, bs = 1, cur = 0, prev = 0;
      do {
        if ((uint32_t)P & bs) {
          prev = cur;
          cur = bs;
          offset -= bs;
          if (blockSize != 0) {
            larger = cur;
            break;
          }
          if (offset <= (uint32_t)rank) {
            blockOff = offset;
            blockSize = cur;
            smaller = prev;
          }
        }
        bs <<= 1;
      } while (offset != 0);
      S = ilog2(blockSize);
      rankInBlock = (uint32_t)rank % blockSize;
    }
    sendOff.assign(S, 0);
    recvOff.assign(S, 0);
    sendCnt.assign(S, 0);
    recvCnt.assign(S, 0);
    stepChunk.assign(S, 0);
    int64_t sc = chunkSize << (steps - 1), so = 0, ro = 0;  // :107-151
    uint32_t bit = 1;
    for (uint32_t i = 0; i < S; i++) {
      const int dest = rank ^ (int)bit;
      stepChunk[i] = sc;
      sendOff[i] = so + ((dest & bit) ? sc : 0);
      recvOff[i] = ro + ((rank & bit) ? sc : 0);
      if (sendOff[i] < count) sendCnt[i] = std::min(sc, count - sendOff[i]);
      if (recvOff[i] < count) recvCnt[i] = std::min(sc, count - recvOff[i]);
      if (rank & bit) {
        so += sc;
        ro += sc;
      }
      bit <<= 1;
      sc >>= 1;
    }
    stepChunkAfter = sc;
    if (smaller != 0) {  // :159-176
      smallerPeer = (int)(blockOff + blockSize + rankInBlock % smaller);
    }
    totalToSend = S > 0 ? recvCnt[S - 1] : count;  // :193-194
    if (larger != 0) {                              // :177-221
      const uint32_t n = larger / blockSize;
      sendCountToLarger = stepChunkAfter >> (ilog2(n) - 1);
      const uint32_t srcOrd = reverseBits(rankInBlock, ilog2(blockSize));
      uint32_t dstOrd = srcOrd * n;
      const uint32_t offLarger = blockOff - larger;
      for (uint32_t k = 0; k < n; k++, dstOrd++) {
        largerPeers.push_back((int)(offLarger + reverseBits(dstOrd, ilog2(larger))));
      }
    }
    // our own receive-region layout
    int64_t at = 0;
    for (uint32_t i = 0; i < S; i++) {
      regionStep.push_back(at);
      at += stepChunk[i] + kPadElems;
    }
    regionSmaller = at;
    if (smaller != 0 && S > 0) at += recvCnt[S - 1] + kPadElems;
    for (size_t k = 0; k < largerPeers.size(); k++) {
      regionLarger.push_back(at);
      at += sendCountToLarger + kPadElems;
    }
    scratch = at;
  }

  // length of the k-th piece sent up to the larger block (0 = not sent)
  int64_t largerPieceLen(size_t k) const {
    if (sendCountToLarger * (int64_t)k >= totalToSend) return 0;
    return std::min(sendCountToLarger, totalToSend - sendCountToLarger * (int64_t)k);
  }
};

}  // namespace

Plan planHalvingDoubling(int rank, int size, int64_t count) {
  Plan p;
  if (count == 0 || size == 1) return p;  // :93-95, :225-241
  const HdGeom g(size, rank, count);
  p.scratch_elems = g.scratch;
  const uint32_t S = g.S;

  // reduce-scatter within the block (:244-259)
  for (uint32_t i = 0; i < S; i++) {
    const int dest = rank ^ (1 << i);
    if (g.sendOff[i] < count) {
      p.steps.push_back({SEND, dest, 0, g.sendOff[i], g.sendCnt[i], 0,
                         HdGeom(size, dest, count).regionStep[i], 0});
      p.bytes_sent += g.sendCnt[i];
    }
    if (g.recvOff[i] < count) {
      p.steps.push_back({RECV, dest, 0, 0, g.recvCnt[i], g.regionStep[i], 0, 0});
      p.steps.push_back({REDUCE, 0, 0, g.recvOff[i], g.recvCnt[i], g.regionStep[i], 0, 0});
      p.steps.push_back({RELEASE, dest, 0, 0, 0, 0, 0, 0});
    }
  }
  // receive from the smaller block (:266-272)
  if (g.smaller != 0 && S > 0 && g.recvCnt[S - 1] > 0) {
    const int from = g.smallerPeer;
    p.steps.push_back({RECV, from, 0, 0, g.recvCnt[S - 1], g.regionSmaller, 0, 0});
    p.steps.push_back({REDUCE, 0, 0, g.recvOff[S - 1], g.recvCnt[S - 1], g.regionSmaller, 0, 0});
    p.steps.push_back({RELEASE, from, 0, 0, 0, 0, 0, 0});
  }
  // scatter to the larger block, then gather its results (:274-305)
  if (g.larger != 0 && g.totalToSend != 0) {
    const int64_t offset = S > 0 ? g.recvOff[S - 1] : 0;
    for (size_t k = 0; k < g.largerPeers.size(); k++) {
      const int64_t len = g.largerPieceLen(k);
      if (len == 0) continue;
      const int to = g.largerPeers[k];
      const HdGeom gt(size, to, count);
      if (gt.smallerPeer != rank || gt.S == 0 || gt.recvCnt[gt.S - 1] != len) {
        fail("halving-doubling cross-block send/recv mismatch");
      }
      p.steps.push_back({SEND, to, 0, offset + (int64_t)k * g.sendCountToLarger, len, 0,
                         gt.regionSmaller, 0});
      p.bytes_sent += len;
    }
    for (size_t k = 0; k < g.largerPeers.size(); k++) {
      const int64_t len = g.largerPieceLen(k);
      if (len == 0) continue;
      const int from = g.largerPeers[k];
      p.steps.push_back({RECV, from, 0, 0, len, g.regionLarger[k], 0, 0});
      p.steps.push_back({COPY, 0, 0, offset + (int64_t)k * g.sendCountToLarger, len,
                         g.regionLarger[k], 0});
      p.steps.push_back({RELEASE, from, 0, 0, 0, 0, 0, 0});
    }
  }
  // send to the smaller block (:308-316)
  if (g.smaller != 0 && S > 0 && g.recvOff[S - 1] < count) {
    const int to = g.smallerPeer;
    const HdGeom gt(size, to, count);
    size_t k = 0;
    while (k < gt.largerPeers.size() && gt.largerPeers[k] != rank) k++;
    if (k == gt.largerPeers.size() || gt.largerPieceLen(k) != g.recvCnt[S - 1]) {
      fail("halving-doubling smaller-block send mismatch");
    }
    p.steps.push_back({SEND, to, 0, g.recvOff[S - 1], g.recvCnt[S - 1], 0,
                       gt.regionLarger[k], 0});
    p.bytes_sent += g.recvCnt[S - 1];
  }
  // allgather within the block, reverse order (:319-341)
  for (uint32_t ii = S; ii-- > 0;) {
    const int dest = rank ^ (1 << ii);
    if (g.recvOff[ii] < count) {
      p.steps.push_back({SEND, dest, 0, g.recvOff[ii], g.recvCnt[ii], 0,
                         HdGeom(size, dest, count).regionStep[ii], 0});
      p.bytes_sent += g.recvCnt[ii];
    }
    if (g.sendOff[ii] < count) {
      p.steps.push_back({RECV, dest, 0, 0, g.sendCnt[ii], g.regionStep[ii], 0, 0});
      p.steps.push_back({COPY, 0, 0, g.sendOff[ii], g.sendCnt[ii], g.regionStep[ii], 0, 0});
      p.steps.push_back({RELEASE, dest, 0, 0, 0, 0, 0, 0});
    }
  }
  return p;
}

// ---------------------------------------------------------------------------
// Owner-computes over the full xGMI mesh
// ---------------------------------------------------------------------------
// A ring reduces each owner's range along a chain of ranks, every rank
// computing op(its value, partial) in place.  Here the owner receives the
// other ranks' copies of its range directly (P-1 copies on P-1 different
// links) and evaluates the same chain in one FOLD; then it sends the
// finished range to every rank (the allgather as one all-to-all round).
// chain(c) lists the ranks of owner c's chain in FOLD order (s[0] first).
namespace {

template <typename Range, typename Chain>
Plan meshPlan(int rank, int size, Range range, Chain chain) {
  Plan p;
  int64_t maxLen = 0;
  for (int c = 0; c < size; c++) {
    int64_t off, len;
    range(c, &off, &len);
    maxLen = std::max(maxLen, len);
  }
  const int64_t region = maxLen + kPadElems;
  // scratch: [0, P) reduce-scatter regions by source rank, [P, 2P) results
  p.scratch_elems = 2 * (int64_t)size * region;
  int64_t myOff, myLen;
  range(rank, &myOff, &myLen);
  for (int d = 1; d < size; d++) {  // my copy of range j to its owner j
    const int j = (rank + d) % size;
    int64_t off, len;
    range(j, &off, &len);
    if (len == 0) continue;
    p.steps.push_back({SEND, j, 0, off, len, 0, (int64_t)rank * region, 0});
    p.bytes_sent += len;
  }
  if (myLen > 0) {
    const std::vector<int> order = chain(rank);
    std::vector<int64_t> srcs;
    for (int from : order) {
      if (from == rank) {
        srcs.push_back(-1);  // our own copy is ptr0 itself
        continue;
      }
      p.steps.push_back({RECV, from, 0, 0, myLen, (int64_t)from * region, 0, 0});
      srcs.push_back((int64_t)from * region);
    }
    p.folds.push_back(srcs);
    p.steps.push_back({FOLD, -1, (int64_t)srcs.size(), myOff, myLen,
                       (int64_t)p.folds.size() - 1, 0, 0});
    for (int from : order) {
      if (from != rank) p.steps.push_back({RELEASE, from, 0, 0, 0, 0, 0, 0});
    }
    for (int d = 1; d < size; d++) {  // the finished range to everyone
      const int j = (rank + d) % size;
      p.steps.push_back({SEND, j, 1, myOff, myLen, 0, (int64_t)(size + rank) * region, 0});
      p.bytes_sent += myLen;
    }
  }
  for (int d = 1; d < size; d++) {
    const int k = (rank - d + size) % size;
    int64_t off, len;
    range(k, &off, &len);
    if (len == 0) continue;
    p.steps.push_back({RECV, k, 1, 0, len, (int64_t)(size + k) * region, 0, 0});
    p.steps.push_back({COPY, 0, 0, off, len, (int64_t)(size + k) * region, 0, 0});
    p.steps.push_back({RELEASE, k, 1, 0, 0, 0, 0, 0});
  }
  return p;
}

}  // namespace

// Replicated: every rank folds every owner's range from all P copies.
template <typename Range, typename Chain>
Plan replicatedPlan(int rank, int size, int64_t count, Range range, Chain chain) {
  Plan p;
  const int64_t region = count + kPadElems;
  p.scratch_elems = (int64_t)size * region;  // one whole-buffer region per source rank
  for (int d = 1; d < size; d++) {
    const int j = (rank + d) % size;
    p.steps.push_back({SEND, j, 2, 0, count, 0, (int64_t)rank * region, 0});
    p.bytes_sent += count;
  }
  for (int d = 1; d < size; d++) {
    const int k = (rank - d + size) % size;
    p.steps.push_back({RECV, k, 2, 0, count, (int64_t)k * region, 0, 0});
  }
  for (int c = 0; c < size; c++) {
    int64_t off, len;
    range(c, &off, &len);
    if (len == 0) continue;
    std::vector<int64_t> srcs;
    for (int from : chain(c)) srcs.push_back(from == rank ? -1 : (int64_t)from * region);
    p.folds.push_back(srcs);
    p.steps.push_back({FOLD, -1, (int64_t)srcs.size(), off, len,
                       (int64_t)p.folds.size() - 1, 0, kFoldWhole});
  }
  for (int d = 1; d < size; d++) {
    p.steps.push_back({RELEASE, (rank - d + size) % size, 2, 0, 0, 0, 0, 0});
  }
  return p;
}

// AllreduceRing (gloo/allreduce_ring.h:81-110): round k hands rank r the
// locally reduced buffer of rank r-1-k (forwarded by the ranks between), and
// ptrs[0] = op(ptrs[0], inbox) (:94): a left fold over r, r-1, ..., r-P+1.
Plan planRing(int rank, int size, int64_t count) {
  if (count == 0 || size == 1) return Plan();
  Plan p;
  const int64_t region = count + kPadElems;
  p.scratch_elems = (int64_t)size * region;  // one whole-buffer region per source rank
  for (int d = 1; d < size; d++) {
    const int j = (rank + d) % size;
    p.steps.push_back({SEND, j, 2, 0, count, 0, (int64_t)rank * region, 0});
    p.bytes_sent += count;
  }
  std::vector<int64_t> srcs = {-1};  // acc = ptrs[0] (the local fold)
  for (int d = 1; d < size; d++) {
    const int k = (rank - d + size) % size;
    p.steps.push_back({RECV, k, 2, 0, count, (int64_t)k * region, 0, 0});
    srcs.push_back((int64_t)k * region);
  }
  p.folds.push_back(srcs);
  p.steps.push_back({FOLD, -1, (int64_t)srcs.size(), 0, count, 0, 0, kFoldLeft | kFoldWhole});
  for (int d = 1; d < size; d++) {
    p.steps.push_back({RELEASE, (rank - d + size) % size, 2, 0, 0, 0, 0, 0});
  }
  return p;
}

// AllreduceBcube's geometry (gloo/allreduce_bcube.h:620-695 setupNodes /
// updateGroupNodes, :150-240 Node / Group): per rank and step its peers (in
// group order), and the [offset, offset + count) it reduces and later sends.
namespace {

struct ClassBcubeGeom {
  int steps = 0;
  std::vector<std::vector<std::vector<int>>> peers;  // [rank][step]
  std::vector<std::vector<int64_t>> num, off;        // [rank][step]

  ClassBcubeGeom(int nodes, int base, int64_t total) {
    // computeSteps (:514-519): float logs, as the reference computes them
    const float lg2n = (float)std::log2((double)nodes);
    const float lg2p = (float)std::log2((double)base);
    const float q = lg2n / lg2p;
    steps = (int)std::ceil(q);
    peers.assign((size_t)nodes, std::vector<std::vector<int>>((size_t)steps));
    num.assign((size_t)nodes, std::vector<int64_t>((size_t)steps, 0));
    off.assign((size_t)nodes, std::vector<int64_t>((size_t)steps, 0));
    int64_t peerDistance = 1;
    for (int step = 0; step < steps; ++step) {
      for (int first = 0; first < nodes; ++first) {
        if (!peers[(size_t)first][(size_t)step].empty()) continue;  // not a group's first node
        std::vector<int> ranks;  // Group::getNodeRanks
        for (int i = 0; i < base; ++i) {
          const int64_t pr = first + i * peerDistance;
          if (pr < nodes) ranks.push_back((int)pr);
        }
        int64_t ptrOffset = step == 0 ? 0 : off[(size_t)first][(size_t)step - 1];
        const int64_t groupCount = step == 0 ? total : num[(size_t)first][(size_t)step - 1];
        const int64_t numElems = std::max<int64_t>(groupCount, (int64_t)ranks.size());
        const int64_t sz = (int64_t)ranks.size();  // updateGroupNodes
        int64_t cnt = numElems / sz;
        const int64_t rem = numElems % sz;
        if (cnt == 0) cnt = 1;
        for (int64_t i = 0; i < sz; ++i) {
          const size_t n = (size_t)ranks[(size_t)i];
          for (int pr : ranks) {
            if (pr != (int)n) peers[n][(size_t)step].push_back(pr);
          }
          const int64_t c = i != sz - 1 ? cnt : cnt + rem;
          num[n][(size_t)step] = c;
          off[n][(size_t)step] = ptrOffset;
          ptrOffset = (ptrOffset + c) % total;
        }
      }
      peerDistance *= base;
    }
  }
};

}  // namespace

Plan planBcube(int rank, int size, int64_t count, int base) {
  if (base < 2) fail("bcube: base must be at least 2");
  if (count == 0 || size == 1) return Plan();  // :273-275, :343-351
  const ClassBcubeGeom g(size, base, count);
  Plan p;
  // receive regions: one per (step, peer index), sized to the largest
  // message (:289-296 size them max(mine, theirs) per pair)
  int64_t maxLen = 0;
  for (int r = 0; r < size; r++)
    for (int s = 0; s < g.steps; s++) maxLen = std::max(maxLen, g.num[(size_t)r][(size_t)s]);
  const int64_t region = maxLen + kPadElems;
  const int perStep = base - 1;
  p.scratch_elems = (int64_t)g.steps * perStep * region;
  auto regionOf = [&](int receiver, int sender, int step) -> int64_t {
    const auto& ps = g.peers[(size_t)receiver][(size_t)step];
    for (size_t i = 0; i < ps.size(); i++) {
      if (ps[i] == sender) return ((int64_t)step * perStep + (int64_t)i) * region;
    }
    fail("bcube: sender is not a peer of the receiver at this step");
    return 0;
  };
  const auto& myPeers = g.peers[(size_t)rank];
  // reduce-scatter (:354-381): sends first, then every peer's message folded
  // into my range in group order
  for (int s = 0; s < g.steps; ++s) {
    for (int dest : myPeers[(size_t)s]) {
      const int64_t n = g.num[(size_t)dest][(size_t)s];
      p.steps.push_back({SEND, dest, 0, g.off[(size_t)dest][(size_t)s], n, 0,
                         regionOf(dest, rank, s), 0});
      p.bytes_sent += n;
    }
    for (int src : myPeers[(size_t)s]) {
      const int64_t n = g.num[(size_t)rank][(size_t)s];
      const int64_t at = regionOf(rank, src, s);
      p.steps.push_back({RECV, src, 0, 0, n, at, 0, 0});
      p.steps.push_back({REDUCE, 0, 0, g.off[(size_t)rank][(size_t)s], n, at, 0, 0});
      p.steps.push_back({RELEASE, src, 0, 0, 0, 0, 0, 0});
    }
  }
  // all-gather (:386-418): the steps in reverse, my range out, theirs in
  for (int s = g.steps - 1; s >= 0; --s) {
    for (int dest : myPeers[(size_t)s]) {
      const int64_t n = g.num[(size_t)rank][(size_t)s];
      p.steps.push_back({SEND, dest, 0, g.off[(size_t)rank][(size_t)s], n, 0,
                         regionOf(dest, rank, s), 0});
      p.bytes_sent += n;
    }
    for (int src : myPeers[(size_t)s]) {
      const int64_t n = g.num[(size_t)src][(size_t)s];
      const int64_t at = regionOf(rank, src, s);
      p.steps.push_back({RECV, src, 0, 0, n, at, 0, 0});
      p.steps.push_back({COPY, 0, 0, g.off[(size_t)src][(size_t)s], n, at, 0, 0});
      p.steps.push_back({RELEASE, src, 0, 0, 0, 0, 0, 0});
    }
  }
  return p;
}

// ring_chunked (gloo/allreduce_ring_chunked.h:106-158) reduces chunk pair j
// (chunks 2j, 2j+1) along ranks j, j+1, ..., j+P-1: rank j+k computes
// op(x[j+k], partial) in place.  The broadcast pass (:163-200) becomes the
// all-to-all round.
Plan planRingChunkedMesh(int rank, int size, int64_t count) {
  if (count == 0 || size == 1) return Plan();
  const int64_t chunks = 2 * (int64_t)size;
  const int64_t chunkSize = std::max<int64_t>(256, (count + chunks - 1) / chunks);
  auto pair = [&](int j, int64_t* off, int64_t* len) {
    int64_t o = 2 * (int64_t)j * chunkSize;
    *off = o;
    *len = o < count ? std::min(2 * chunkSize, count - o) : 0;
  };
  auto chain = [&](int j) {
    std::vector<int> v;
    for (int k = 0; k < size; k++) v.push_back((j + k) % size);
    return v;
  };
  return meshPlan(rank, size, pair, chain);
}

Plan planRingChunkedReplicated(int rank, int size, int64_t count) {
  if (count == 0 || size == 1) return Plan();
  const int64_t chunks = 2 * (int64_t)size;
  const int64_t chunkSize = std::max<int64_t>(256, (count + chunks - 1) / chunks);
  auto pair = [&](int j, int64_t* off, int64_t* len) {
    int64_t o = 2 * (int64_t)j * chunkSize;
    *off = o;
    *len = o < count ? std::min(2 * chunkSize, count - o) : 0;
  };
  auto chain = [&](int j) {
    std::vector<int> v;
    for (int k = 0; k < size; k++) v.push_back((j + k) % size);
    return v;
  };
  return replicatedPlan(rank, size, count, pair, chain);
}

// ---------------------------------------------------------------------------
// gloo::allreduce(opts), Algorithm::RING (gloo/allreduce.cc:148-393)
// ---------------------------------------------------------------------------
namespace {

struct FnRingGeom {
  int64_t count = 0, chunkE = 0, npc = 0, pieceE = 0, S = 0;

  // piece g (mod S): owner chunk g / npc, piece g % npc within it; the
  // length is clipped to the buffer and may be 0 (the reference's
  // out-of-range segments, :256-262).
  void piece(int64_t g, int64_t* off, int64_t* len) const {
    g %= S;
    const int64_t c = g / npc, j = g % npc;
    const int64_t o = c * chunkE + j * pieceE;
    int64_t l = std::max<int64_t>(0, std::min(pieceE, chunkE - j * pieceE));
    l = o < count ? std::min(l, count - o) : 0;
    *off = o;
    *len = l;
  }
};

int64_t roundUp(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

FnRingGeom fnRingGeom(int size, int64_t count, const PlanParams& prm) {
  const int64_t es = prm.esize;
  if (es <= 0) fail("element size must be positive");
  const int64_t P = size;
  const int64_t totalBytes = count * es;
  // :193-219 (maxSegmentBytes, numSegments, segmentBytes)
  const int64_t maxSegmentBytes = es * std::max<int64_t>(1, prm.maxSegmentBytes / es);
  const int64_t numSegments = roundUp(
      std::max((totalBytes + maxSegmentBytes - 1) / maxSegmentBytes, 2 * P), P);
  const int64_t spr = numSegments / P;
  const int64_t segmentBytes = roundUp((totalBytes + numSegments - 1) / numSegments, es);
  const int64_t segE = segmentBytes / es;
  FnRingGeom g;
  g.count = count;
  // Rank c ends the reduce-scatter owning segments [c*spr, (c+1)*spr): the
  // element range [c*chunkE, (c+1)*chunkE).  That ownership (and the chain
  // c-1, c-2, ..., c along which it is reduced) fixes every result bit; the
  // pieces it is moved in do not.
  g.chunkE = spr * segE;
  const int64_t target = std::max(segE, prm.minPieceBytes / es);
  // >= 2 pieces per chunk keeps the reference's invariant that a piece is
  // reduced before it is forwarded (spr >= 2, :214-216)
  g.npc = std::max<int64_t>(2, (g.chunkE + target - 1) / target);
  g.npc = std::min(g.npc, spr);
  g.pieceE = (g.chunkE + g.npc - 1) / g.npc;
  g.S = P * g.npc;
  return g;
}

}  // namespace

Plan planFnRing(int rank, int size, int64_t count, const PlanParams& prm) {
  Plan p;
  if (count == 0 || size == 1) return p;  // :98-100, :129-133
  const FnRingGeom g = fnRingGeom(size, count, prm);
  const int64_t region = g.pieceE + kPadElems;
  // tmp (two segments, :221-232) for the reduce-scatter; the allgather
  // receives into out directly in the reference (:382), here via two more
  // regions and a COPY
  p.scratch_elems = 4 * region;
  const int recvRank = (rank + 1) % size;         // :158
  const int sendRank = (rank + size - 1) % size;  // :159
  const int64_t iters = g.S - g.npc + 2;          // :264-279
  // reduce/scatter (:279-322)
  for (int64_t i = 0; i < iters; i++) {
    if (i >= 2) {
      const int64_t k = i - 2;
      int64_t off, len;
      g.piece((rank + 2) * (int64_t)g.npc + k, &off, &len);  // recvOffset, :252-254
      if (len > 0) {
        const int64_t ch = k & 1;
        p.steps.push_back({RECV, recvRank, ch, 0, len, ch * region, 0, 0});
        p.steps.push_back({REDUCE, 0, 0, off, len, ch * region, 0, 0});
        p.steps.push_back({RELEASE, recvRank, ch, 0, 0, 0, 0, 0});
      }
    }
    if (i < g.S - g.npc) {
      int64_t off, len;
      g.piece((rank + 1) * (int64_t)g.npc + i, &off, &len);  // sendOffset, :249-251
      if (len > 0) {
        const int64_t ch = i & 1;
        p.steps.push_back({SEND, sendRank, ch, off, len, 0, ch * region, 0});
        p.bytes_sent += len;
      }
    }
  }
  // allgather (:362-392)
  for (int64_t i = 0; i < iters; i++) {
    if (i >= 2) {
      const int64_t k = i - 2;
      int64_t off, len;
      g.piece((rank + 1) * (int64_t)g.npc + k, &off, &len);  // recvOffset, :336-338
      if (len > 0) {
        const int64_t ch = 2 + (k & 1);
        p.steps.push_back({RECV, recvRank, ch, 0, len, ch * region, 0, 0});
        p.steps.push_back({COPY, 0, 0, off, len, ch * region, 0, 0});
        p.steps.push_back({RELEASE, recvRank, ch, 0, 0, 0, 0, 0});
      }
    }
    if (i < g.S - g.npc) {
      int64_t off, len;
      g.piece((int64_t)rank * g.npc + i, &off, &len);  // sendOffset, :333-335
      if (len > 0) {
        const int64_t ch = 2 + (i & 1);
        p.steps.push_back({SEND, sendRank, ch, off, len, 0, ch * region, 0});
        p.bytes_sent += len;
      }
    }
  }
  return p;
}

Plan planFnRingMesh(int rank, int size, int64_t count, const PlanParams& prm) {
  if (count == 0 || size == 1) return Plan();
  const FnRingGeom g = fnRingGeom(size, count, prm);
  auto range = [&](int c, int64_t* off, int64_t* len) {
    const int64_t o = (int64_t)c * g.chunkE;
    *off = o;
    *len = o < count ? std::min(g.chunkE, count - o) : 0;
  };
  // chunk c starts at rank c-1 (:313-318) and moves leftward, each rank
  // computing op(its value, partial) (:286-297), ending at rank c
  auto chain = [&](int c) {
    std::vector<int> v;
    for (int k = 1; k <= size; k++) v.push_back((c - k + 2 * size) % size);
    return v;
  };
  return meshPlan(rank, size, range, chain);
}

Plan planFnRingReplicated(int rank, int size, int64_t count, const PlanParams& prm) {
  if (count == 0 || size == 1) return Plan();
  const FnRingGeom g = fnRingGeom(size, count, prm);
  auto range = [&](int c, int64_t* off, int64_t* len) {
    const int64_t o = (int64_t)c * g.chunkE;
    *off = o;
    *len = o < count ? std::min(g.chunkE, count - o) : 0;
  };
  auto chain = [&](int c) {
    std::vector<int> v;
    for (int k = 1; k <= size; k++) v.push_back((c - k + 2 * size) % size);
    return v;
  };
  return replicatedPlan(rank, size, count, range, chain);
}

// ---------------------------------------------------------------------------
// gloo::allreduce(opts), Algorithm::BCUBE (gloo/allreduce.cc:395-669)
// ---------------------------------------------------------------------------
namespace {

struct BcubeGroup {
  int64_t bufferOffset = 0, bufferLength = 0, chunkLength = 0;
  int64_t myChunkOffset = 0, myChunkLength = 0;
  int groupRank = 0;
  std::vector<int> ranks;
  int64_t slot = 0;    // receive slot size (elements) for one member
  int64_t rsBase = 0;  // receive regions of this step: member i at base + i * slot
  int64_t agBase = 0;

  int64_t len(int i) const {  // :545-550
    return std::min(chunkLength, std::max<int64_t>(0, bufferLength - i * chunkLength));
  }
};

struct BcubeGeom {
  std::vector<BcubeGroup> groups;
  int64_t scratch = 0;

  BcubeGeom(int rank, int size, int64_t count) {
    // computeGroupSizePerStep(size, 2), :398-409
    std::vector<int64_t> sizes;
    int64_t rest = size;
    while (rest % 2 == 0) {
      sizes.push_back(2);
      rest /= 2;
    }
    if (rest > 1) sizes.push_back(rest);
    int64_t peerDistance = 1, bufferOffset = 0, bufferLength = count;
    for (int64_t gs : sizes) {  // :466-511
      BcubeGroup g;
      g.groupRank = (int)((rank / peerDistance) % gs);
      const int64_t base = rank - g.groupRank * peerDistance;
      for (int64_t i = 0; i < gs; i++) g.ranks.push_back((int)(base + i * peerDistance));
      g.bufferOffset = bufferOffset;
      g.bufferLength = bufferLength;
      g.chunkLength = (bufferLength + gs - 1) / gs;
      g.myChunkOffset = bufferOffset + g.groupRank * g.chunkLength;
      g.myChunkLength = g.len(g.groupRank);
      groups.push_back(g);
      peerDistance *= gs;
      bufferOffset = g.myChunkOffset;
      bufferLength = g.myChunkLength;
    }
    int64_t at = 0;
    for (auto& g : groups) {
      g.slot = g.chunkLength + kPadElems;
      g.rsBase = at;
      at += (int64_t)g.ranks.size() * g.slot;
      g.agBase = at;
      at += (int64_t)g.ranks.size() * g.slot;
    }
    scratch = at;
  }
};

}  // namespace

Plan planFnBcube(int rank, int size, int64_t count) {
  Plan p;
  if (count == 0 || size == 1) return p;
  const BcubeGeom geo(rank, size, count);
  p.scratch_elems = geo.scratch;
  std::vector<BcubeGeom> peerGeo;  // receivers' region layouts
  peerGeo.reserve((size_t)size);
  for (int r = 0; r < size; r++) peerGeo.emplace_back(r, size, count);
  const size_t nsteps = geo.groups.size();
  // reduce/scatter (:520-597)
  for (size_t s = 0; s < nsteps; s++) {
    const BcubeGroup& g = geo.groups[s];
    for (size_t i = 0; i < g.ranks.size(); i++) {  // :534-556
      const int dst = g.ranks[i];
      if (dst == rank) continue;
      const int64_t len = g.len((int)i);
      if (len == 0) continue;  // the peer's receive is empty too
      const BcubeGroup& pg = peerGeo[(size_t)dst].groups[s];
      p.steps.push_back({SEND, dst, 0, g.bufferOffset + (int64_t)i * g.chunkLength, len, 0,
                         pg.rsBase + (int64_t)g.groupRank * pg.slot, 0});
      p.bytes_sent += len;
    }
    if (g.myChunkLength == 0) continue;
    std::vector<int64_t> srcs{-1};
    for (size_t i = 0; i < g.ranks.size(); i++) {  // :521-532
      const int src = g.ranks[i];
      if (src == rank) continue;
      const int64_t region = g.rsBase + (int64_t)i * g.slot;
      p.steps.push_back({RECV, src, 0, 0, g.myChunkLength, region, 0, 0});
      srcs.push_back(region);
    }
    // out = op(out, tmp[i]) for the peers in group order (:580-596)
    if (srcs.size() == 2) {
      p.steps.push_back({REDUCE, 0, 0, g.myChunkOffset, g.myChunkLength, srcs[1], 0, 0});
    } else {
      p.folds.push_back(srcs);
      p.steps.push_back({FOLD, -1, (int64_t)srcs.size(), g.myChunkOffset, g.myChunkLength,
                         (int64_t)p.folds.size() - 1, 0, kFoldLeft});
    }
    for (size_t i = 0; i < g.ranks.size(); i++) {
      if (g.ranks[i] != rank) p.steps.push_back({RELEASE, g.ranks[i], 0, 0, 0, 0, 0, 0});
    }
  }
  // allgather, groups in reverse (:606-669)
  for (size_t s = nsteps; s-- > 0;) {
    const BcubeGroup& g = geo.groups[s];
    if (g.myChunkLength > 0) {
      for (size_t i = 0; i < g.ranks.size(); i++) {
        const int dst = g.ranks[i];
        if (dst == rank) continue;
        const BcubeGroup& pg = peerGeo[(size_t)dst].groups[s];
        p.steps.push_back({SEND, dst, 1, g.myChunkOffset, g.myChunkLength, 0,
                           pg.agBase + (int64_t)g.groupRank * pg.slot, 0});
        p.bytes_sent += g.myChunkLength;
      }
    }
    for (size_t i = 0; i < g.ranks.size(); i++) {
      const int src = g.ranks[i];
      if (src == rank) continue;
      const int64_t len = g.len((int)i);
      if (len == 0) continue;
      const int64_t region = g.agBase + (int64_t)i * g.slot;
      p.steps.push_back({RECV, src, 1, 0, len, region, 0, 0});
      p.steps.push_back({COPY, 0, 0, g.bufferOffset + (int64_t)i * g.chunkLength, len, region, 0});
      p.steps.push_back({RELEASE, src, 1, 0, 0, 0, 0, 0});
    }
  }
  return p;
}

int autoRingSchedule(int size, int64_t bytes, bool fn, bool deviceDriven) {
  const int ring = fn ? ALGO_FN_RING : ALGO_RING_CHUNKED;
  const int mesh = fn ? ALGO_FN_RING_MESH : ALGO_RING_CHUNKED_MESH;
  const int repl = fn ? ALGO_FN_RING_REPL : ALGO_RING_CHUNKED_REPL;
  // host-mediated: the reference's kOnDeviceThreshold (algorithm.cc:16).
  // Device-driven: one-shot moves S per link in one round, two-shot 2S/P per
  // link in two; with a round costing L and links B, one-shot wins below
  // S* = L·B / (1 - 2/P): always at P = 2, ~1-2 MiB at P = 4, less at P = 8.
  int64_t maxRepl = int64_t(256) << 10;
  if (deviceDriven) {
    maxRepl = size <= 2 ? (int64_t(16) << 20) : size <= 4 ? (int64_t(2) << 20)
                                                          : (int64_t(1) << 20);
  }
  if (size <= 1) return ring;
  if (bytes <= maxRepl) return repl;
  // the mesh lands about S per rank in one block (the two-shot's slot
  // arrays; 2S/P regions on the steps engines), and a block shared between
  // processes stays below 2 GiB (Context::kIpcMaxBlockBytes): larger
  // buffers take the ring, whose regions are S/2P (class) or 4 MiB pieces
  // (function-style)
  return bytes < kMeshMaxBytes ? mesh : ring;
}

namespace {
// GLOO_AMD_MAX_MESSAGE_BYTES sets the initial value (tests: split programs at
// small sizes in every rank process)
std::atomic<int64_t> g_maxMessageBytes{[] {
  const char* e = std::getenv("GLOO_AMD_MAX_MESSAGE_BYTES");
  const int64_t v = e != nullptr ? std::atoll(e) : 0;
  return v >= 4096 ? v : kMaxMessageBytes;
}()};
}  // namespace

int64_t maxMessageBytes() { return g_maxMessageBytes.load(); }

void setMaxMessageBytes(int64_t bytes) {
  g_maxMessageBytes.store(bytes > 0 ? bytes : kMaxMessageBytes);
}

void splitMessages(Plan& p, int64_t M, int64_t V, bool forward) {
  if (M <= 0 || V <= 0 || M % V != 0) fail("splitMessages: bad piece length");
  for (const Step& s : p.steps) {
    if (s.kind == FOLD && (s.flags & kFoldWhole) != 0) return;  // left whole (plan.h)
  }
  // A message for [off, off + len) lands at its region's 16-byte base plus
  // the phase ph = off mod V; sub-region q of the region is [qM, (q+1)M)
  // past that base, so piece q holds the message's elements
  // [off - ph + qM, off - ph + (q+1)M) clipped to it: every piece after the
  // first starts at phase 0 exactly at its sub-region's base, and the
  // sub-regions are the same for every message of the region.
  auto pieces = [&](int64_t off, int64_t len) {  // (no overflow for any M)
    const int64_t span = off % V + len;
    return span <= M ? (int64_t)1 : (span - 1) / M + 1;
  };
  auto piece = [&](int64_t off, int64_t len, int64_t q, int64_t* o, int64_t* l) {
    if (off % V + len <= M) {  // one piece (and no (q + 1) * M to overflow)
      *o = off;
      *l = len;
      return;
    }
    const int64_t a = q == 0 ? off : off - off % V + q * M;
    const int64_t b = std::min(off + len, off - off % V + (q + 1) * M);
    *o = a;
    *l = std::max<int64_t>(0, b - a);
  };
  std::vector<Step> out;
  out.reserve(p.steps.size() * 2);
  const std::vector<Step>& in = p.steps;
  for (size_t i = 0; i < in.size();) {
    const Step& s = in[i];
    if (s.kind == SEND) {
      for (int64_t q = 0; q < pieces(s.off, s.len); q++) {
        Step t = s;
        t.channel = s.channel + q * kPieceChannelStride;
        piece(s.off, s.len, q, &t.off, &t.len);
        t.dst_off = s.dst_off + q * M;
        out.push_back(t);
      }
      i++;
      continue;
    }
    if (s.kind != RECV) {
      out.push_back(s);
      i++;
      continue;
    }
    // a receive group: RECVs, the steps reading their regions, and their
    // RELEASEs, up to the RELEASE that leaves no message of the group
    // unreleased (every schedule's shape)
    std::map<int64_t, int64_t> region;                    // region -> its message's length
    std::map<int64_t, int64_t> regionOff;                 // region -> its message's offset
    std::map<std::pair<int64_t, int64_t>, int64_t> open;  // (peer, channel) -> region
    std::vector<int64_t> released;                        // per group step: RELEASE's region
    size_t j = i;
    for (; j < in.size(); j++) {
      const Step& t = in[j];
      released.push_back(-1);
      if (t.kind == RECV) {
        region[t.boff] = t.len;
        open[{t.peer, t.channel}] = t.boff;
      } else if (t.kind == RELEASE) {
        auto it = open.find({t.peer, t.channel});
        if (it == open.end()) fail("splitMessages: a RELEASE without its RECV in the group");
        released.back() = it->second;
        open.erase(it);
        if (open.empty()) break;
      } else if (t.kind == SEND) {
        fail("splitMessages: a SEND inside a receive group");
      }
    }
    if (j == in.size()) fail("splitMessages: a receive group without its RELEASE");
    // the receiver learns a message's offset from the steps that read it
    auto reads = [&](int64_t boff, int64_t off, int64_t len) {
      auto it = region.find(boff);
      if (it == region.end() || it->second != len) {
        fail("splitMessages: a step reads a region other than its group's whole message");
      }
      auto ot = regionOff.find(boff);
      if (ot != regionOff.end() && ot->second != off) {
        fail("splitMessages: two steps read one message at different offsets");
      }
      regionOff[boff] = off;
    };
    for (size_t k = i; k <= j; k++) {
      const Step& t = in[k];
      if (t.kind == REDUCE || t.kind == COPY) reads(t.boff, t.off, t.len);
      if (t.kind == FOLD) {
        for (int64_t r : p.folds[(size_t)t.boff]) {
          if (r >= 0) reads(r, t.off, t.len);
        }
      }
    }
    auto piecesOf = [&](int64_t boff) {
      const int64_t len = region.at(boff);
      if (len == 0) return (int64_t)1;
      auto ot = regionOff.find(boff);
      if (ot == regionOff.end()) fail("splitMessages: a message no step reads");
      return pieces(ot->second, len);
    };
    int64_t K = 1;
    for (const auto& kv : region) K = std::max(K, piecesOf(kv.first));
    // the SENDs right after the group forwarding one of its results, sent
    // per piece inside the loop below (forward)
    size_t fwdEnd = j + 1;
    if (forward) {
      while (fwdEnd < in.size() && in[fwdEnd].kind == SEND && in[fwdEnd].len > 0) {
        bool result = false;
        for (size_t k = i; k <= j; k++) {
          result = result || ((in[k].kind == REDUCE || in[k].kind == COPY ||
                               in[k].kind == FOLD) &&
                              in[k].off == in[fwdEnd].off && in[k].len == in[fwdEnd].len);
        }
        if (!result) break;
        fwdEnd++;
      }
    }
    for (size_t f = j + 1; f < fwdEnd; f++) K = std::max(K, pieces(in[f].off, in[f].len));
    for (int64_t q = 0; q < K; q++) {
      for (size_t k = i; k <= j; k++) {
        const Step& t = in[k];
        Step u = t;
        if (t.kind == RECV) {
          if (q >= piecesOf(t.boff)) continue;
          int64_t o = 0;
          if (t.len > 0) piece(regionOff.at(t.boff), t.len, q, &o, &u.len);
          u.channel = t.channel + q * kPieceChannelStride;
          u.boff = t.boff + q * M;
        } else if (t.kind == RELEASE) {
          if (q >= piecesOf(released[k - i])) continue;
          u.channel = t.channel + q * kPieceChannelStride;
        } else if (t.kind == REDUCE || t.kind == COPY) {
          if (q >= piecesOf(t.boff)) continue;
          piece(t.off, t.len, q, &u.off, &u.len);
          u.boff = t.boff + q * M;
        } else if (t.kind == FOLD) {
          const int64_t n = pieces(t.off, t.len);
          if (q >= n) continue;
          std::vector<int64_t> srcs;
          for (int64_t r : p.folds[(size_t)t.boff]) srcs.push_back(r < 0 ? r : r + q * M);
          if (n > 1) {
            p.folds.push_back(srcs);
            u.boff = (int64_t)p.folds.size() - 1;
          }
          piece(t.off, t.len, q, &u.off, &u.len);
        }
        out.push_back(u);
      }
      for (size_t f = j + 1; f < fwdEnd; f++) {  // the forwards of piece q
        const Step& t = in[f];
        if (q >= pieces(t.off, t.len)) continue;
        Step u = t;
        u.channel = t.channel + q * kPieceChannelStride;
        piece(t.off, t.len, q, &u.off, &u.len);
        u.dst_off = t.dst_off + q * M;
        out.push_back(u);
      }
    }
    i = fwdEnd;
  }
  p.steps = std::move(out);
}

namespace {
std::atomic<int64_t> g_pipelineBytes{[] {
  const char* e = std::getenv("GLOO_AMD_PIPELINE_BYTES");
  const int64_t v = e != nullptr ? std::atoll(e) : 0;
  return v >= 4096 ? v : (int64_t)0;
}()};
}  // namespace

int64_t pipelineBytes() { return g_pipelineBytes.load(); }

void setPipelineBytes(int64_t bytes) { g_pipelineBytes.store(bytes >= 4096 ? bytes : 0); }

Plan makePlan(int algo, int rank, int size, int64_t count, const PlanParams& prm) {
  if (size < 1 || rank < 0 || rank >= size || count < 0) fail("bad geometry");
  Plan p;
  switch (algo) {
    case ALGO_RING_CHUNKED: p = planRingChunked(rank, size, count); break;
    case ALGO_HALVING_DOUBLING: p = planHalvingDoubling(rank, size, count); break;
    case ALGO_RING_CHUNKED_MESH: p = planRingChunkedMesh(rank, size, count); break;
    case ALGO_FN_RING: p = planFnRing(rank, size, count, prm); break;
    case ALGO_FN_RING_MESH: p = planFnRingMesh(rank, size, count, prm); break;
    case ALGO_FN_BCUBE: p = planFnBcube(rank, size, count); break;
    case ALGO_RING_CHUNKED_REPL: p = planRingChunkedReplicated(rank, size, count); break;
    case ALGO_FN_RING_REPL: p = planFnRingReplicated(rank, size, count, prm); break;
    case ALGO_RING: p = planRing(rank, size, count); break;
    case ALGO_BCUBE: p = planBcube(rank, size, count, prm.base); break;
    default: fail("unknown algorithm");
  }
  // pieces of a whole number of 16-byte vectors (the landing phase rule)
  const int64_t es = std::max(1, prm.esize);
  const int64_t V = 16 / std::min<int64_t>(16, es);
  int64_t bytesPer = prm.maxMessageBytes;
  if (prm.pipelineBytes > 0) bytesPer = std::min(bytesPer, prm.pipelineBytes);
  const int64_t M = std::max<int64_t>(V, bytesPer / es / V * V);
  splitMessages(p, M, V, prm.pipelineBytes > 0);
  return p;
}

// ---------------------------------------------------------------------------
// The plan kernel's segments, channels and message numbers
// ---------------------------------------------------------------------------
namespace {

bool dataStep(const Step& s) {
  return (s.kind == SEND && s.len > 0) || s.kind == REDUCE || s.kind == COPY || s.kind == FOLD;
}

int chanOf(std::vector<std::pair<int, int>>& v, int peer, int tag) {
  for (size_t i = 0; i < v.size(); i++) {
    if (v[i].first == peer && v[i].second == tag) return (int)i;
  }
  v.emplace_back(peer, tag);
  return (int)v.size() - 1;
}

// See SyncTable::safe.  Byte ownership of message [a, a+len) in its landing
// region: element x sits at byte (a*es mod 16) + (x - a)*es and belongs to
// workgroup w when it lies in slice w of its segment.
bool regionsSafe(const std::vector<Plan>& all, const std::vector<int64_t>& bounds, int64_t sl,
                 int G, int es) {
  struct Iv {
    int64_t b0, b1;
    int w;
  };
  auto owners = [&](int64_t a, int64_t len) {
    std::vector<Iv> v;
    const int64_t ph = (a * es) % 16;
    auto it = std::upper_bound(bounds.begin(), bounds.end(), a) - 1;
    for (; it + 1 != bounds.end() && *it < a + len; ++it) {
      const int64_t s0 = *it, s1 = *(it + 1);
      for (int w = 0; w < G; w++) {
        const int64_t x = std::max(a, s0 + (int64_t)w * sl);
        const int64_t y = std::min(std::min(a + len, s1), s0 + (int64_t)(w + 1) * sl);
        if (x < y) v.push_back({ph + (x - a) * es, ph + (y - a) * es, w});
      }
    }
    std::sort(v.begin(), v.end(), [](const Iv& p, const Iv& q) { return p.b0 < q.b0; });
    return v;
  };
  auto agree = [](const std::vector<Iv>& m, const std::vector<Iv>& n) {
    size_t i = 0, j = 0;
    while (i < m.size() && j < n.size()) {
      const int64_t lo = std::max(m[i].b0, n[j].b0), hi = std::min(m[i].b1, n[j].b1);
      if (lo < hi && m[i].w != n[j].w) return false;
      if (m[i].b1 < n[j].b1) {
        i++;
      } else {
        j++;
      }
    }
    return true;
  };
  const int size = (int)all.size();
  for (int q = 0; q < size; q++) {
    // the messages landing in each of q's regions: the k-th RECV of (p, tag)
    // is the k-th SEND of p to q on tag
    std::map<int64_t, std::vector<std::pair<int64_t, int64_t>>> byRegion;
    std::map<std::pair<int, int>, int> nrecv;
    for (const auto& s : all[(size_t)q].steps) {
      if (s.kind != RECV) continue;
      const int p = (int)s.peer, tag = (int)s.channel;
      const int k = nrecv[{p, tag}]++;
      const Step* snd = nullptr;
      int seen = 0;
      for (const auto& u : all[(size_t)p].steps) {
        if (u.kind == SEND && u.peer == q && u.channel == tag && seen++ == k) {
          snd = &u;
          break;
        }
      }
      if (snd == nullptr) return false;  // programs disagree: never run the kernel on them
      if (snd->len == 0) continue;
      auto& v = byRegion[s.boff];
      const std::pair<int64_t, int64_t> m{snd->off, snd->len};
      if (std::find(v.begin(), v.end(), m) == v.end()) v.push_back(m);
    }
    for (const auto& kv : byRegion) {
      const auto& ms = kv.second;
      std::vector<std::vector<Iv>> own;
      for (const auto& m : ms) own.push_back(owners(m.first, m.second));
      for (size_t i = 0; i < ms.size(); i++) {
        for (size_t j = i + 1; j < ms.size(); j++) {
          if (!agree(own[i], own[j])) return false;
        }
      }
    }
  }
  return true;
}

}  // namespace

int64_t landedRegionElems(const Plan& plan, int64_t start, int64_t next) {
  int64_t longest = -1;
  for (const auto& s : plan.steps) {
    if (s.kind == RECV && s.boff == start) longest = std::max(longest, s.len);
  }
  return longest < 0 ? 0 : std::min(next - start, longest + kPadElems);
}

int64_t maxRegionOf(const Plan& plan) {
  std::vector<int64_t> starts{0, plan.scratch_elems};
  for (const auto& s : plan.steps) {
    if (s.kind == RECV) starts.push_back(s.boff);
  }
  std::sort(starts.begin(), starts.end());
  starts.erase(std::unique(starts.begin(), starts.end()), starts.end());
  int64_t m = 0;  // over the regions some message lands in (the executor's blocks)
  for (size_t i = 0; i + 1 < starts.size(); i++) {
    m = std::max(m, landedRegionElems(plan, starts[i], starts[i + 1]));
  }
  return m;
}

SyncTable syncTable(int algo, int rank, int size, int64_t count, const PlanParams& prm,
                    int G) {
  SyncTable t;
  t.bounds = {0, count};
  Plan mine;
  std::vector<Plan> all;
  for (int q = 0; q < size; q++) {
    Plan p = makePlan(algo, q, size, count, prm);
    for (const auto& s : p.steps) {
      if (!dataStep(s)) continue;
      if (s.off < 0 || s.off + s.len > count) fail("sync table: step range outside the buffer");
      t.bounds.push_back(s.off);
      t.bounds.push_back(s.off + s.len);
    }
    if (q == rank) mine = p;
    t.maxRegionElems = std::max(t.maxRegionElems, maxRegionOf(p));
    all.push_back(std::move(p));
  }
  std::sort(t.bounds.begin(), t.bounds.end());
  t.bounds.erase(std::unique(t.bounds.begin(), t.bounds.end()), t.bounds.end());
  if (G < 1) fail("sync table: G must be >= 1");
  const int64_t V = 16 / std::max(1, prm.esize);
  int64_t maxSeg = 1;
  for (size_t k = 0; k + 1 < t.bounds.size(); k++) {
    maxSeg = std::max(maxSeg, t.bounds[k + 1] - t.bounds[k]);
  }
  t.slice = ((maxSeg + G - 1) / G + V - 1) / V * V;
  t.safe = regionsSafe(all, t.bounds, t.slice, G, prm.esize);
  auto segIndex = [&](int64_t x) {
    auto it = std::lower_bound(t.bounds.begin(), t.bounds.end(), x);
    if (it == t.bounds.end() || *it != x) fail("sync table: not a segment bound");
    return (int32_t)(it - t.bounds.begin());
  };
  std::vector<uint64_t> sent, recvd, released;
  t.steps.resize(mine.steps.size());
  for (size_t i = 0; i < mine.steps.size(); i++) {
    const Step& s = mine.steps[i];
    StepSync& y = t.steps[i];
    if (s.kind == SEND) {
      y.chan = chanOf(t.outChans, (int)s.peer, (int)s.channel);
      sent.resize(t.outChans.size());
      y.seq = ++sent[(size_t)y.chan];
    } else if (s.kind == RECV) {
      y.chan = chanOf(t.inChans, (int)s.peer, (int)s.channel);
      recvd.resize(t.inChans.size());
      y.seq = ++recvd[(size_t)y.chan];
    } else if (s.kind == RELEASE) {
      y.chan = chanOf(t.inChans, (int)s.peer, (int)s.channel);
      released.resize(t.inChans.size());
      y.seq = ++released[(size_t)y.chan];
    }
    if (dataStep(s)) {
      y.seg0 = segIndex(s.off);
      y.seg1 = segIndex(s.off + s.len);
    }
  }
  recvd.resize(t.inChans.size());
  released.resize(t.inChans.size());
  if (recvd != released) fail("sync table: RECV and RELEASE counts differ");
  for (size_t i = 0; i < mine.steps.size(); i++) {
    const Step& s = mine.steps[i];
    StepSync& y = t.steps[i];
    if (s.kind == SEND) y.perRun = sent[(size_t)y.chan];
    if (s.kind == RECV || s.kind == RELEASE) y.perRun = recvd[(size_t)y.chan];
  }
  // the message a REDUCE / COPY reads: the latest RECV into its region
  {
    std::map<int64_t, size_t> lastRecv;  // region -> step
    for (size_t i = 0; i < mine.steps.size(); i++) {
      const Step& s = mine.steps[i];
      if (s.kind == RECV) lastRecv[s.boff] = i;
      if ((s.kind == REDUCE || s.kind == COPY) && s.len > 0) {
        auto it = lastRecv.find(s.boff);
        if (it == lastRecv.end()) fail("sync table: a step reads a region nothing was received into");
        t.steps[i].rseq = t.steps[it->second].seq;
        t.steps[i].rperRun = t.steps[it->second].perRun;
      }
    }
  }
  // two landing slots per channel when no program folds and every landing
  // region is fed by one channel (a region shared by channels would need
  // their slots kept in step)
  t.slots = 2;
  for (const Plan& p : all) {
    std::map<int64_t, std::pair<int64_t, int64_t>> feeder;  // region -> (peer, channel)
    for (const Step& s : p.steps) {
      if (s.kind == FOLD) {
        t.slots = 1;
        t.anyFold = true;
      }
      if (s.kind != RECV) continue;
      auto it = feeder.find(s.boff);
      const std::pair<int64_t, int64_t> ch{s.peer, s.channel};
      if (it == feeder.end()) {
        feeder[s.boff] = ch;
      } else if (it->second != ch) {
        t.slots = 1;
      }
    }
  }
  // reduce-and-forward: a REDUCE / COPY followed (past RELEASEs only) by the
  // SEND of exactly its range (only with two slots: see plan.h)
  for (size_t i = 0; i < mine.steps.size() && t.slots == 2; i++) {
    const Step& s = mine.steps[i];
    if ((s.kind != REDUCE && s.kind != COPY) || s.len <= 0) continue;
    size_t j = i + 1;
    while (j < mine.steps.size() && mine.steps[j].kind == RELEASE) j++;
    if (j < mine.steps.size() && mine.steps[j].kind == SEND && mine.steps[j].off == s.off &&
        mine.steps[j].len == s.len && t.steps[j].fuse < 0) {
      t.steps[i].fuse = (int32_t)j;
      t.steps[j].fuse = (int32_t)i;
    }
  }
  // partial reduce-and-forward: the SEND after a REDUCE / COPY (past
  // RELEASEs only) overlaps its range without equalling it (plan.h "pre")
  for (size_t i = 0; i < mine.steps.size() && t.slots == 2; i++) {
    const Step& s = mine.steps[i];
    if ((s.kind != REDUCE && s.kind != COPY) || s.len <= 0 || t.steps[i].fuse >= 0) continue;
    size_t j = i + 1;
    while (j < mine.steps.size() && mine.steps[j].kind == RELEASE) j++;
    if (j >= mine.steps.size()) continue;
    const Step& u = mine.steps[j];
    if (u.kind != SEND || u.len <= 0 || t.steps[j].fuse >= 0 || t.steps[j].pre >= 0) continue;
    const int64_t lo = std::max(s.off, u.off), hi = std::min(s.off + s.len, u.off + u.len);
    if (lo >= hi) continue;
    t.steps[i].pre = (int32_t)j;
    t.steps[j].pre = (int32_t)i;
    t.steps[i].pre0 = t.steps[j].pre0 = segIndex(lo);
    t.steps[i].pre1 = t.steps[j].pre1 = segIndex(hi);
  }
  // a fused REDUCE's own copy of its result (of the overlap, for a partial
  // one) is dead when the range is next overwritten whole by a COPY before
  // anything reads it (plan.h)
  for (size_t i = 0; i < mine.steps.size(); i++) {
    const Step& s = mine.steps[i];
    const StepSync& y = t.steps[i];
    if (s.kind != REDUCE || (y.fuse < 0 && y.pre < 0)) continue;
    const int64_t lo = y.fuse >= 0 ? s.off : t.bounds[(size_t)y.pre0];
    const int64_t hi = y.fuse >= 0 ? s.off + s.len : t.bounds[(size_t)y.pre1];
    for (size_t k = (size_t)(y.fuse >= 0 ? y.fuse : y.pre) + 1; k < mine.steps.size(); k++) {
      const Step& u = mine.steps[k];
      if (u.kind == RECV || u.kind == RELEASE || u.len <= 0) continue;
      if (u.off >= hi || u.off + u.len <= lo) continue;  // disjoint
      if (u.kind == COPY && u.off <= lo && u.off + u.len >= hi) t.steps[i].keep = 0;
      break;  // the first step touching the range decides
    }
  }
  return t;
}

// ---------------------------------------------------------------------------
// Geometry of the device-driven engines
// ---------------------------------------------------------------------------
namespace {

// slices: >= 4 KiB, a whole number of 16-byte vectors, at most maxSlices
void sliceUp(DeviceLayout& d, int64_t len, int esize, int64_t maxSlices) {
  const int64_t V = 16 / esize, minSlice = 4096 / esize;
  const int64_t gmax = std::max<int64_t>(1, std::min<int64_t>(maxSlices, 1 << 20));
  int64_t slice = (len + gmax - 1) / gmax;
  slice = (std::max(slice, minSlice) + V - 1) / V * V;
  d.slice = slice;
  d.G = (int)std::max<int64_t>(1, (len + slice - 1) / slice);
}

// FOLD sources are region offsets (multiples of `region`) or -1 (ptr0)
void chainOf(const std::vector<int64_t>& f, int64_t region, int rank, int size, int* out) {
  if ((int)f.size() != size) fail("device layout: fold of " + std::to_string(f.size()) +
                                  " sources for " + std::to_string(size) + " ranks");
  for (int i = 0; i < size; i++) {
    const int64_t r = f[(size_t)i];
    if (r >= 0 && r % region != 0) fail("device layout: unexpected fold source");
    out[i] = r < 0 ? rank : (int)(r / region);
  }
}

}  // namespace

DeviceLayout oneShotLayout(const Plan& plan, int rank, int size, int64_t count, int esize,
                           int64_t maxSlices) {
  if (size < 2 || size > kDevMaxRanks || count <= 0) fail("device layout: bad geometry");
  DeviceLayout d;
  sliceUp(d, count, esize, maxSlices);
  const int64_t region = count + kPadElems;  // replicatedPlan's regions
  for (const auto& st : plan.steps) {
    if (st.kind != FOLD) continue;
    if (d.njobs >= kDevMaxRanks) fail("device layout: too many chunk ranges");
    chainOf(plan.folds[(size_t)st.boff], region, rank, size, d.chain[d.njobs]);
    d.jobOff[d.njobs] = st.off;
    d.jobLen[d.njobs] = st.len;
    d.njobs++;
  }
  d.maxLen = count;
  return d;
}

DeviceLayout twoShotLayout(const Plan& plan, int rank, int size, int64_t count, int esize,
                           int64_t maxSlices) {
  if (size < 2 || size > kDevMaxRanks || count <= 0) fail("device layout: bad geometry");
  DeviceLayout d;
  // channel-0 SENDs carry this rank's copy of range j to owner j; the FOLD
  // is our own range.  Every non-empty range is one or the other, so maxLen
  // is the plan's largest range (meshPlan's region = maxLen + pad).
  for (int i = 0; i < size; i++) d.myChain[i] = i;
  const Step* fold = nullptr;
  for (const auto& st : plan.steps) {
    if (st.kind == SEND && st.channel == 0) {
      d.rangeOff[st.peer] = st.off;
      d.rangeLen[st.peer] = st.len;
      d.maxLen = std::max(d.maxLen, st.len);
    } else if (st.kind == FOLD) {
      fold = &st;
    }
  }
  if (fold != nullptr) {
    d.rangeOff[rank] = fold->off;
    d.rangeLen[rank] = fold->len;
    d.maxLen = std::max(d.maxLen, fold->len);
    chainOf(plan.folds[(size_t)fold->boff], d.maxLen + kPadElems, rank, size, d.myChain);
  }
  sliceUp(d, std::max<int64_t>(1, d.maxLen), esize, maxSlices);
  return d;
}

// ---------------------------------------------------------------------------
// Staging of host-memory buffers
// ---------------------------------------------------------------------------
namespace {

// A set of disjoint element intervals.
class IntervalSet {
 public:
  // the parts of [off, off+len) not in the set, ascending
  std::vector<Range> missing(int64_t off, int64_t len) const {
    std::vector<Range> out;
    int64_t at = off;
    const int64_t end = off + len;
    for (const auto& r : v_) {
      if (r.off + r.len <= at) continue;
      if (r.off >= end) break;
      if (r.off > at) out.push_back({at, r.off - at});
      at = std::max(at, r.off + r.len);
      if (at >= end) break;
    }
    if (at < end) out.push_back({at, end - at});
    return out;
  }
  void add(int64_t off, int64_t len) {
    if (len <= 0) return;
    std::vector<Range> nv;
    int64_t lo = off, hi = off + len;
    bool placed = false;
    for (const auto& r : v_) {
      if (r.off + r.len < lo) {
        nv.push_back(r);
      } else if (r.off > hi) {
        if (!placed) nv.push_back({lo, hi - lo});
        placed = true;
        nv.push_back(r);
      } else {
        lo = std::min(lo, r.off);
        hi = std::max(hi, r.off + r.len);
      }
    }
    if (!placed) nv.push_back({lo, hi - lo});
    v_.swap(nv);
  }

 private:
  std::vector<Range> v_;  // sorted, disjoint, non-adjacent
};

bool writes(const Step& s) { return s.kind == REDUCE || s.kind == COPY || s.kind == FOLD; }
bool touches(const Step& s) { return (s.kind == SEND || writes(s)) && s.len > 0; }

}  // namespace

StagePlan stagePlan(const Plan& plan, int64_t count, int64_t maxPiece) {
  StagePlan sp;
  if (maxPiece <= 0) maxPiece = count > 0 ? count : 1;
  IntervalSet issued;
  auto issue = [&](int64_t off, int64_t len) {
    for (const Range& r : issued.missing(off, len)) {
      for (int64_t at = r.off; at < r.off + r.len; at += maxPiece) {
        sp.h2d.push_back({at, std::min(maxPiece, r.off + r.len - at)});
      }
      issued.add(r.off, r.len);
    }
  };
  for (const Step& s : plan.steps) {
    if (touches(s)) issue(s.off, s.len);
  }
  issue(0, count);
  sp.d2h.resize(plan.steps.size());
  IntervalSet later;  // written by a later step
  for (size_t i = plan.steps.size(); i-- > 0;) {
    const Step& s = plan.steps[i];
    if (!writes(s) || s.len <= 0) continue;
    sp.d2h[i] = later.missing(s.off, s.len);
    later.add(s.off, s.len);
  }
  sp.d2hRest = later.missing(0, count);
  return sp;
}

}  // namespace glx
