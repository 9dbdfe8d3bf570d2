// merge_schedule.h -- the point-to-point message lists of the co-located merge (comm.hip): the
// payload exchange (every rank's packed rows to their destination ranks) and the gather of the
// reduced partitions to rank 0.  Free of HIP and RCCL, so the host test suite compiles this
// same code and checks that the lists of every (sender, receiver) pair match message for
// message (tests/test_merge_schedule.py): RCCL matches grouped ncclSend / ncclRecv with one
// peer in posting order, and a count or order mismatch would hang or corrupt the exchange.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace bqg_sched {

struct P2P {
  int peer;
  void* ptr;
  size_t bytes;
};

// Exchange: rank r sends its rows for destination d (to_peer[d] of them) column by column
// from src_of(d, j), and receives from every source s (from_peer[s] rows) column by column
// into dst[j] at the rows before s's block (sources in rank order).  to_peer / from_peer are
// rows of the all-gathered [W x W] count matrix, so sender r's to_peer[d] is receiver d's
// from_peer[r].  Self messages (d == r) are posted too (one path for every rank).
template <typename SrcOf>
void exchange_schedule(int W, int ncols, const std::vector<int>& lg, const std::vector<int64_t>& to_peer,
                       const std::vector<int64_t>& from_peer, SrcOf src_of, const std::vector<void*>& dst,
                       std::vector<P2P>& sends, std::vector<P2P>& recvs) {
  for (int d = 0; d < W; ++d) {
    if (!to_peer[d]) continue;
    for (int j = 0; j < ncols; ++j) sends.push_back(P2P{d, src_of(d, j), (size_t)to_peer[d] << lg[j]});
  }
  int64_t off = 0;
  for (int s = 0; s < W; ++s) {
    if (!from_peer[s]) continue;
    for (int j = 0; j < ncols; ++j)
      recvs.push_back(P2P{s, (unsigned char*)dst[j] + ((size_t)off << lg[j]), (size_t)from_peer[s] << lg[j]});
    off += from_peer[s];
  }
}

// Gather: every rank r > 0 sends its part_rows[r] reduced rows to rank 0 column by column from
// src[j]; rank 0 receives them into dst[j] after its own part_rows[0] rows, in rank order.
inline void gather_schedule(int rank, int W, int ncols, const std::vector<int>& lg, const std::vector<int64_t>& part_rows,
                            const std::vector<void*>& src, const std::vector<void*>& dst, std::vector<P2P>& sends,
                            std::vector<P2P>& recvs) {
  if (rank != 0) {
    for (int j = 0; part_rows[rank] && j < ncols; ++j)
      sends.push_back(P2P{0, src[j], (size_t)part_rows[rank] << lg[j]});
    return;
  }
  int64_t off = part_rows[0];
  for (int s = 1; s < W; ++s) {
    if (!part_rows[s]) continue;
    for (int j = 0; j < ncols; ++j)
      recvs.push_back(P2P{s, (unsigned char*)dst[j] + ((size_t)off << lg[j]), (size_t)part_rows[s] << lg[j]});
    off += part_rows[s];
  }
}

}  // namespace bqg_sched
