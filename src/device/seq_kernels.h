// Sequential-chain device kernels: the shared argument block, constants and small device
// helpers, and the declarations of the kernels the DeviceTreeLearner launches. The kernels
// live in four translation units:
//   seq_hist_kernels.hip       gradient quantizer, root sums, k_hist (LDS fixed-point
//                              histograms), slab reduce, owner push and the xGMI exchange
//   seq_scan_kernels.hip       k_reduce_scan (slab fold / owner rows -> threshold scans)
//   seq_vote_kernels.hip       voting-parallel local scan, election, elected-histogram scan
//   seq_partition_kernels.hip  best-leaf select, stable partition, post-split bookkeeping,
//                              score-update traversal, row -> column transpose
// The frontier engine (frontier.h / frontier_kernels.hip) has its own argument block.
#pragma once

#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <string>
#include <vector>
#include "device/grad_kernels.h"
#include "device/hip_common.h"
#include "device/leaf_kernels.h"
#include "device/runtime_internal.h"
#include "device/frontier.h"
#include "device/traverse_kernels.h"
#include "device/sample_kernels.h"
#include "device/split_scan.h"
#include "device/tree_kernels.h"
#include "learner/forced_splits.h"
#include "learner/serial_tree_learner.h"
#include "lgap/common.h"
#include "lgap/device_api.h"
#include "lgap/network.h"
#include "lgap/objective.h"
#include "lgap/rank_math.h"
#include "lgap/split_math.h"

namespace lgap {
namespace device {
namespace seq {

#ifndef LGAP_HIST_THREADS
#define LGAP_HIST_THREADS 512
#endif
#ifndef LGAP_SCAN_UNROLL
#define LGAP_SCAN_UNROLL 8  // slab rows in flight per lane in the k_reduce_scan fold
#endif
#ifndef LGAP_HIST_R
#define LGAP_HIST_R 16
#endif
constexpr int kHistThreads = LGAP_HIST_THREADS;
constexpr int kHistMinRows = 1024;  // A/B on MI355X: 1024 beats 2048 / 512 / 4096 at 1.25M and 10M rows
constexpr int kHistLdsBytes = 56 * 1024;
constexpr int kPartThreads = 256;
constexpr int kPartIters = 16;  // rows per thread of the two-kernel partition (k_part_count / k_part_scatter)
constexpr int kTileRows = kPartThreads * kPartIters;
constexpr int kScanWaves = 4;
#ifndef LGAP_SCAN_FOLD
#define LGAP_SCAN_FOLD 1  // 1: half-wave row streams, one value per lane; 2: quarter-wave streams, value pairs
#endif
#ifndef LGAP_SCAN_THREADS
#define LGAP_SCAN_THREADS 1024  // k_reduce_scan block size (the fold and the slot update use all waves)
#endif
constexpr int kScanThreads = LGAP_SCAN_THREADS;
constexpr int kNodeThreads = 256;

struct Args {
  const uint32_t* rowbins;
  const uint8_t* colbins;
  const float2* gh;
  int* idx[5];  // 0/1 ping-pong (frontier: depth buffers 0, 1), 2 bag, 3/4 frontier depth buffers 2, 3
  int N, stride_dw, width, num_groups, TB, F, L, max_tiles;
  const int* gstart;
  const DevFeature* feat;
  const HistTile* tiles;
  const uint8_t* used_bytree;
  const uint8_t* bynode;
  const TreeParams* tp;
  Ctl* ctl;       // control block this launch reads (never written while the launch runs)
  Ctl* ctl_next;  // k_partition writes the post-split control block here (double buffer)
  LeafRange* range;
  double2* lsum;
  double* lout;
  int* gcount;
  int* depth;
  int* slot;
  LeafBounds* bounds;
  SplitInfo* best;
  SplitRec* rec;
  double* slots;
  double* staging;
  float* staging_f;  // data-parallel all-reduce row of the fp32 (default) histogram path
  void* hist_slab;
  unsigned* ghmax;  // float bits of max|g|, max|h|, sum|g|, sum|h| over the root rows
  uint8_t* splittable;
  int* tile_cnt;
  int* tile_off;
  unsigned* rng;
  int max_cat_bin;
  int max_bin;  // largest feature num_bin (LDS sizing of k_reduce_scan)
  int cat_p2;   // power of two >= the largest categorical num_bin (categorical sort scratch), 1 without
  char* scan_scratch;        // global-memory scan scratch (features wider than the LDS budget), else null
  size_t scan_scratch_stride;  // bytes per block
  int max_depth;
  int fuse_post;
  unsigned long long* stamps;  // optional phase timestamps (LGAP_STAMPS=1)
  int distributed;
  int use_monotone;
  double monotone_penalty;
  double cegb_split;  // cegb_tradeoff * cegb_penalty_split (per row of the leaf), 0: none
  // interaction constraints: bit k of ic_feat[f] = constraint set k holds f;
  // ic_leaf[leaf] = sets that hold every feature on the leaf's branch
  const unsigned long long* ic_feat;
  unsigned long long* ic_leaf;
  double* root_part;  // per-block (sum g, sum h, max|g|, max|h|, sum|g|, sum|h|) of k_root_sums
  unsigned* bar;      // {-, -, error flag of k_partition's bounded waits}
  SplitKey* leaf_key;  // [L] compact best split per leaf (next to best)
  unsigned long long* tile_pub;  // k_partition tile counts tagged with the split epoch
  int hist_min_rows;  // rows per k_hist block (fewer rows: more blocks and slab rows)
  // ---- owner-computes split finding (tree_learner=data|feature); single GPU: P = 1, Fmax = F
  int P, rank, Fmax;  // ranks, this rank, candidate block width (most features any rank owns)
  int cand_rows;        // blocks of the candidate table the select reads (P for data / feature parallel)
  const int* own_feat;  // [Fmax] features of the groups this rank owns (-1: padding); nullptr: identity
  char* cand;           // candidate table [P] blocks of cand_stride bytes (tree_kernels.h)
  int cand_stride;
  int cand_key_bytes;   // SplitKey part of a block (SplitInfo part follows)
  int scan_src;         // 0: fold the k_hist slab rows; 1: sum the `nparts` owner rows of `rx`
  // split slab fold (scan_src 0): fold_chunks blocks per feature each fold a run of the slab
  // rows into fold_part; the last to arrive on fold_cnt[j] sums the runs and scans
  int fold_chunks, fold_feats;
  double* fold_part;   // [fold_chunks][2 * TB]
  unsigned* fold_cnt;  // [F]: a multiple of fold_chunks between launches
  const void* rx;       // owner row: the 2 * bbin reduce-scattered values of the bins this rank owns
  int own_bin0;         // first histogram bin this rank owns
  int bbin;             // owner block width (bins, padded to the largest block)
  const int* bin_lo;    // [P + 1] owner bin bounds (k_hist_owner permutation)
  // ---- voting parallel (tree_learner=voting): local scan, top-k vote, elected histograms
  int vote;             // 1: k_reduce_scan is the LOCAL pass (local sums / counts, no masks or penalties)
  double2* hsum_part;   // [hist blocks] local (sum g, sum h) of the smaller child's rows per k_hist block
  double2* lsum_loc;    // [L] local leaf sums
  int topk;             // elected features per child (min(top_k, F))
  const char* lcand;    // local candidate table (keys [2][F], infos [2][F] at lcand_key_bytes)
  int lcand_key_bytes;
  VoteRec* vrec;        // gathered local top-k records [P][2 * topk]
  void* vhist;          // packed elected histograms (all-reduced in place)
  int vcap;             // values of one packed row (2 * topk * 2 * (max_bin - 1))
  int* elect;           // [2][topk + 2]: count, first-value offset, then the elected features (ascending)
  SplitParams sp;
};

__device__ __forceinline__ SplitKey* CandKey(const Args& a, int r, int sel, int j) {
  return reinterpret_cast<SplitKey*>(a.cand + static_cast<size_t>(r) * a.cand_stride) + sel * a.Fmax + j;
}
__device__ __forceinline__ SplitInfo* CandInfo(const Args& a, int r, int sel, int j) {
  return reinterpret_cast<SplitInfo*>(a.cand + static_cast<size_t>(r) * a.cand_stride + a.cand_key_bytes) +
         sel * a.Fmax + j;
}
// full record of the candidate at table position `pos` (SplitKey::pos) of child `sel`
__device__ __forceinline__ SplitInfo* CandInfoPos(const Args& a, int sel, int pos) {
  const int r = pos / a.Fmax;
  return CandInfo(a, r, sel, pos - r * a.Fmax);
}

// ---------------------------------------------------------------------------
// small device helpers

__device__ __forceinline__ uint32_t ColBin(const Args& a, int g, int row) {
  const size_t o = static_cast<size_t>(g) * a.N + row;
  return a.width == 1 ? a.colbins[o] : reinterpret_cast<const uint16_t*>(a.colbins)[o];
}

__device__ __forceinline__ int RowAt(const Args& a, int buf, int pos) { return buf < 0 ? pos : a.idx[buf][pos]; }

// Diagnostic phase stamps: [kernel 0..4][split 0..255][block 0..1][stamp 0..7], 100 MHz wall clock.
__device__ __forceinline__ void Stamp(const Args& a, int kernel, int i) {
  if (a.stamps != nullptr && blockIdx.x < 2 && blockIdx.y == 0 && threadIdx.x == 0) {
    const int split = a.ctl->num_splits & 255;
    a.stamps[((static_cast<size_t>(kernel) * 256 + split) * 2 + blockIdx.x) * 8 + i] = wall_clock64();
  }
}
// Latest exit over all blocks of a kernel (slot 0, stamp 7), for kernel-span / gap analysis.
__device__ __forceinline__ void StampEnd(const Args& a, int kernel) {
  if (a.stamps != nullptr && threadIdx.x == 0) {
    const int split = a.ctl->num_splits & 255;
    atomicMax(&a.stamps[((static_cast<size_t>(kernel) * 256 + split) * 2) * 8 + 7], wall_clock64());
  }
}
// A stamp of a given block role (slot 0) for a given split, with an explicit clock value.
__device__ __forceinline__ void StampAt(const Args& a, int kernel, int split, int i, unsigned long long v) {
  if (a.stamps != nullptr && threadIdx.x == 0) a.stamps[((static_cast<size_t>(kernel) * 256 + (split & 255)) * 2) * 8 + i] = v;
}


constexpr int kRootThreads = 256;
constexpr int kVoteThreads = 256;
constexpr int kTraverseThreads = 256;
constexpr int kTraverseMaxDw = 16;

__device__ __forceinline__ int HistActiveBlocks(int n, int grid, int min_rows) {
  int nb = (n + min_rows - 1) / min_rows;
  return nb > grid ? grid : nb;
}

// seq_hist_kernels.hip
__global__ void k_qmax(const float2* gh, int n, unsigned* qmax);
__global__ void k_quantize(float2* gh, float2* gh_true, uint16_t* ghq, int n, const unsigned* qmax,
                                                  int bins, int const_hess, uint32_t seed, int stochastic);
__global__ void k_init_tree(Args a);
__global__ void k_root_sums(Args a);
__global__ void k_root_final(Args a, int nblocks);
template <int W, int MODE>
__global__ void k_hist(Args a);
template <typename Acc, typename Out>
__global__ void k_hist_reduce(Args a, int hist_grid, Out* __restrict__ out);
template <typename Acc>
__global__ void k_hist_owner(Args a, int hist_grid, Acc* __restrict__ stage);

// seq_scan_kernels.hip
template <typename Acc, bool kGlobal>
__global__ void k_reduce_scan(Args a, int hist_grid);

// seq_vote_kernels.hip
__global__ void k_vote_local(Args a);
template <typename Acc>
__global__ void k_vote_pack(Args a);
template <typename Acc, bool kGlobal>
__global__ void k_vote_scan(Args a);
__global__ void k_leaf_true_sums(Args a, const float2* gh_true, int num_leaves,
                                                                  double2* out);

// seq_partition_kernels.hip
__global__ void k_part_count(Args a);
__global__ void k_part_scatter(Args a);
template <int ITERS>
__global__ void k_partition(Args a);
__global__ void k_post(Args a);
__global__ void k_add_tree(const uint32_t* __restrict__ rowbins, int stride_dw,
                                                               int width, int N, const DevNode* __restrict__ nodes,
                                                               int num_nodes, const uint32_t* __restrict__ cat_bits,
                                                               const double* __restrict__ leaf_value,
                                                               double* __restrict__ score);
template <typename T>
__global__ void k_transpose_bins(const uint32_t* __restrict__ rowbins, int stride_dw, int N, int G,
                                                        uint8_t* __restrict__ colbins);

}  // namespace seq
}  // namespace device
}  // namespace lgap
