// plan.cc -- compile the reference schedules into per-rank step programs.
//
// The element ranges, peers and orders of operations are those of the
// reference algorithms (cited per block); only the buffer management is
// ours: every incoming channel gets its own padded receive region in the
// rank's device scratch, and flow control is per-channel credits instead of
// the reference's separate notification buffers.
#include "plan.h"

#include <algorithm>
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
// ring_chunked semantics over the full xGMI mesh
// ---------------------------------------------------------------------------
// The ring (gloo/allreduce_ring_chunked.h:106-158) reduces chunk pair j
// (chunks 2j, 2j+1) along ranks j, j+1, ..., j+P-1: rank j+k computes
// op(x[j+k], partial) in place.  Here rank j receives x[j+1..j+P-1] of pair j
// directly from each owner (P-1 copies, P-1 different links) and evaluates the
// same chain in one FOLD; then it sends the finished pair to every rank
// (the broadcast pass, :163-200, as one all-to-all round).
Plan planRingChunkedMesh(int rank, int size, int64_t count) {
  Plan p;
  if (count == 0 || size == 1) return p;
  const int64_t chunks = 2 * (int64_t)size;
  const int64_t chunkSize = std::max<int64_t>(256, (count + chunks - 1) / chunks);
  const int64_t region = 2 * chunkSize + kPadElems;
  auto pair = [&](int j, int64_t* off, int64_t* len) {
    int64_t o = 2 * (int64_t)j * chunkSize;
    int64_t l = 0;
    if (o < count) l = std::min(2 * chunkSize, count - o);
    *off = o;
    *len = l;
  };
  // scratch: [0, P) reduce-scatter regions by source rank, [P, 2P) results
  p.scratch_elems = 2 * (int64_t)size * region;
  int64_t myOff, myLen;
  pair(rank, &myOff, &myLen);
  for (int d = 1; d < size; d++) {  // my copy of pair j to its owner j
    const int j = (rank + d) % size;
    int64_t off, len;
    pair(j, &off, &len);
    if (len == 0) continue;
    p.steps.push_back({SEND, j, 0, off, len, 0, (int64_t)rank * region, 0});
    p.bytes_sent += len;
  }
  if (myLen > 0) {
    std::vector<int64_t> srcs{-1};  // x[rank] is ptr0 itself
    for (int k = 1; k < size; k++) {
      const int from = (rank + k) % size;
      p.steps.push_back({RECV, from, 0, 0, myLen, (int64_t)from * region, 0, 0});
      srcs.push_back((int64_t)from * region);
    }
    p.folds.push_back(srcs);
    p.steps.push_back({FOLD, -1, (int64_t)srcs.size(), myOff, myLen,
                       (int64_t)p.folds.size() - 1, 0, 0});
    for (int k = 1; k < size; k++) {
      p.steps.push_back({RELEASE, (rank + k) % size, 0, 0, 0, 0, 0, 0});
    }
    for (int d = 1; d < size; d++) {  // the finished pair to everyone
      const int j = (rank + d) % size;
      p.steps.push_back({SEND, j, 1, myOff, myLen, 0, (int64_t)(size + rank) * region, 0});
      p.bytes_sent += myLen;
    }
  }
  for (int d = 1; d < size; d++) {
    const int k = (rank - d + size) % size;
    int64_t off, len;
    pair(k, &off, &len);
    if (len == 0) continue;
    p.steps.push_back({RECV, k, 1, 0, len, (int64_t)(size + k) * region, 0, 0});
    p.steps.push_back({COPY, 0, 0, off, len, (int64_t)(size + k) * region, 0, 0});
    p.steps.push_back({RELEASE, k, 1, 0, 0, 0, 0, 0});
  }
  return p;
}

Plan makePlan(int algo, int rank, int size, int64_t count) {
  if (size < 1 || rank < 0 || rank >= size || count < 0) fail("bad geometry");
  if (algo == ALGO_RING_CHUNKED) return planRingChunked(rank, size, count);
  if (algo == ALGO_HALVING_DOUBLING) return planHalvingDoubling(rank, size, count);
  if (algo == ALGO_RING_CHUNKED_MESH) return planRingChunkedMesh(rank, size, count);
  fail("unknown algorithm");
  return Plan();
}

}  // namespace glx
