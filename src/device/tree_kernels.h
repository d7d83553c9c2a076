// Device-side state of the HIP tree learner. Everything that changes while a
// tree grows (leaf ranges, best splits, the split about to be applied) lives
// in device memory so the whole leaf-wise growth loop is a fixed sequence of
// kernels with fixed launch shapes: it is captured once into a hipGraph and
// replayed per tree; kernels whose work vanished (tree finished early) exit
// on the `done` flag.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "lgap/split_math.h"

namespace lgap {
namespace device {

struct DevFeature {
  int group;
  int offset;       // first group bin
  int num_bin;
  int mfb;          // most frequent bin (implicit in histograms)
  int default_bin;
  int hist_offset;  // global histogram position of group bin `offset`
  int8_t missing;
  int8_t bin_type;
  int8_t monotone;
  int8_t pad;
  int pad2;
  double penalty;
};

// Histogram tile: a run of whole dwords of the packed row (so whole groups)
// whose bins fit in the LDS budget of one workgroup.
struct HistTile {
  int d0, d1;    // dword range within a row
  int g0, g1;    // groups [g0, g1)
  int bin0;      // global histogram index of the first bin of group g0
  int nbins;     // bins covered
  int direct;    // 1: bins exceed the LDS budget, accumulate in global memory
  int pad;
};

// Rows of a leaf: positions [start, start+count) of index buffer `buf`
// (buf -1: identity order, i.e. all rows without bagging; 2: the bag list).
struct LeafRange {
  int buf, start, count, pad;
};

// Per-tree inputs written by the host before each replay.
struct TreeParams {
  int root_buf;
  int root_count;
  int cls;
  int root_gcount;  // global (all ranks) row count of the root
  float spec_alpha;  // frontier engine: speculation depth, fraction of the remaining budget (host-tuned per tree)
  unsigned byn_rng;  // frontier engine, by-node draws in the select (FArgs::byn_draw): the sampler's state after the root's
  int pad[2];
};

struct Ctl {
  int num_leaves, done, smaller, larger;
  int skip, num_splits, split_leaf, new_leaf;
  int parent_buf, parent_start, parent_count, target_buf;
  int left_count, cls, scan_round, max_count;  // max_count: largest leaf (rows), bounds useful grid size
  int hist_nb;  // slab rows holding the smaller child's histogram when k_partition built it (0: k_hist did)
  unsigned epoch;  // split sequence number (never reset): tags k_partition's published tile counts
  int pad1, pad2;
  double plg, plh;  // voting-parallel: this rank's local (sum g, sum h) of the leaf just split
};

// Compact record of a split candidate: everything the best-leaf select and the
// partition predicate need, written by k_reduce_scan next to each SplitInfo and
// persisted per leaf, so the select is one round of 48-byte loads.
struct SplitKey {
  double gain;  // kMinScore: no split
  int feature;  // -1: no split
  uint32_t threshold;
  int group, offset, num_bin, mfb;
  int default_bin;
  int8_t missing, default_left, is_cat, pad0;
  int pos;  // candidate position (rank * Fmax + owned index): where the full SplitInfo sits
  int pad2;
};

// Owner-computes data parallelism: every rank scans the features of the groups it
// owns and publishes its candidates as one block; the blocks of all ranks form the
// candidate table [P][ SplitKey[2][Fmax] | SplitInfo[2][Fmax] ] that every rank's
// best-leaf select reads (single GPU: P = 1, Fmax = F).
constexpr int kMaxXRanks = 16;  // xGMI transport: ranks of one node

// xGMI transport: each rank's exchange buffer (IPC-mapped, uncached device memory)
// holds [histogram receive rows][candidate table][flags][root rows] at identical
// offsets on every rank; base[q] is rank q's buffer in this process's address space.
struct XPeers {
  char* base[kMaxXRanks];
};

// Voting-parallel: one rank's local top-k candidate of one child (LightSplitInfo,
// split_info.hpp:199-262): best local gain of a feature and its left + right count.
struct VoteRec {
  double gain;
  int feature;  // -1: empty
  int count;
};

struct SplitRec {
  int leaf, left_count, right_count, pad;
  SplitInfo info;
};

// Device-resident tree for score updates (one tree uploaded at a time).
struct DevNode {
  int group, offset, num_bin, mfb;
  int default_bin, missing, threshold, decision;  // decision: bit0 categorical, bit1 default_left
  int left, right, cat_begin, cat_nwords;
};

}  // namespace device
}  // namespace lgap
