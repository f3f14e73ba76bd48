// peer_rule.hpp -- the termination rule of the GPU-initiated peer transport
// (csrc/dymu_dist.cpp PeerTransport::run), kept apart from the HIP
// code so the CPU tests compile and exercise it (tests/test_peer_rule.py).
//
// Every rank posts, at each check c, its status: P (tiles queued for its round's
// first two passes), and per link side (0: to rank-1, 1: to rank+1) S (pushes that
// carried a decrease = the tags it wrote) and R (the smallest tag its merge read).
// The ranks' rounds are not aligned; each rank's check-c status is a snapshot at
// its own check c.  A check is quiet when every rank had P = 0 and every link had
// R = S (the receiver merged the sender's latest push); the solve is done after
// two consecutive quiet checks between which no S moved -- then no push can be in
// flight or unmerged and no rank has work (the four-counter argument).
#pragma once

#include <cstdint>
#include <vector>

namespace dymu_peer {

struct Status {
  uint64_t P = 0, S[2] = {0, 0}, R[2] = {0, 0};
};

// every rank idle and every link's pushes merged, in one check's snapshots
inline bool quiet(const std::vector<Status>& st) {
  for (size_t q = 0; q < st.size(); ++q) {
    if (st[q].P != 0) return false;
    // link q -> q+1: q's pushes to rank+1 (side 1) against q+1's merges from rank-1
    // (side 0), and the reverse direction
    if (q + 1 < st.size() && (st[q].S[1] != st[q + 1].R[0] || st[q + 1].S[0] != st[q].R[1]))
      return false;
  }
  return true;
}

// no rank pushed a decrease between the two checks
inline bool same_pushes(const std::vector<Status>& prev, const std::vector<Status>& cur) {
  for (size_t q = 0; q < cur.size(); ++q)
    if (cur[q].S[0] != prev[q].S[0] || cur[q].S[1] != prev[q].S[1]) return false;
  return true;
}

// the decision at check c from checks c-1 (prev, prev_quiet) and c (cur)
inline bool done(const std::vector<Status>& prev, bool prev_quiet, const std::vector<Status>& cur) {
  return prev_quiet && quiet(cur) && same_pushes(prev, cur);
}

}  // namespace dymu_peer
