// Frontier tree growth: leaf-wise (best-first) trees built in batched ROUNDS.
//
// Leaf-wise growth splits, at every step, the leaf whose best split has the largest
// gain. A leaf's best split is a pure function of its rows, so the split of ANY leaf
// can be computed before best-first order reaches it. The frontier engine exploits
// that: each round expands a batch of open nodes at once (partition their rows,
// histogram their smaller children, parent - smaller subtraction, threshold scans of
// both children), and a replay of the sequential best-first order over the computed
// nodes commits splits in exactly the order (and with exactly the leaf numbering) of
// the one-split-at-a-time learner. A round's batch always holds the node the replay is
// blocked on (the highest-gain unexpanded leaf), plus speculative expansions of the
// next-best open nodes; speculation that the budget (num_leaves) never commits is
// simply dropped. Rounds ~ depth of the tree instead of num_leaves - 1 sequential
// splits, so the per-launch latency floor is paid ~4-5x less often, and each round's
// kernels get several leaves' worth of parallel work.
//
// Per round (all device-resident, fixed launch shapes, replayed from a hipGraph):
//   k_f_partition  stable 2-way partition of every expanded parent's rows (decoupled
//                  look-back per expansion), post-split bookkeeping of the children
//   k_f_hist       LDS fixed-point histograms of every expansion's smaller child,
//                  flushed with integer atomics into one per-expansion accumulator at
//                  the tree's global fixed-point scale (deterministic, no slab)
//   k_f_scan       one workgroup per (expansion, feature): accumulator -> smaller
//                  child's histogram, larger = parent - smaller, both children scanned
//   k_f_select     one workgroup: per-child best split, replay of best-first order,
//                  choice of the next round's expansions
//
// Intermediate monotone constraints (FArgs::mono_inter): a committed split also tightens the
// bounds of leaves elsewhere in the tree (the host's constraint climb), so a leaf's record can go
// stale after it was scanned. The select tracks each leaf's current bounds (cbnd) against the
// ones its record was scanned with (bounds); a stale record is an upper bound of its re-scan, so
// the replay only stops where a stale leaf could still win, and the next round re-scans the stale
// leaves from their histogram slots (FExp::rescan: no tiles, no rows) and voids expansions grown
// from their old records (the subtree dies).
//
// Beyond 256 alive nodes the select does not re-sort the alive list: keys never change once
// computed (outside CEGB re-scoring and monotone rescans), so last round's order (salive) filtered
// to the nodes still alive is merged with the children the round just scanned.
//
// Row lists: a node at depth d >= 1 keeps its row indices in depth buffer (d - 1) % 4
// (the root: the bag or identity order). Children of depth-d nodes never overwrite
// their parent's list, and a speculative expansion is only allowed where the list it
// would overwrite (the ancestor 4 levels up) belongs to an already committed split, so
// every final leaf's list stays intact for the score update and leaf renewal.
//
// Reference parity: serial_tree_learner.cpp:179-245 (Train loop), :477-622
// (FindBestSplitsFromHistograms), :766-922 (SplitInner bookkeeping);
// cuda_single_gpu_tree_learner.cpp:158-345 (the reference's device loop, one split per
// step); data_partition.hpp:101 (Split); leaf numbering of Tree::Split (tree.cpp:61).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device/tree_kernels.h"
#include "lgap/split_math.h"

namespace lgap {
namespace device {

constexpr int kFrontierKmax = 64;   // expansions per round (compile-time cap)
#ifndef LGAP_FRONTIER_BUFS
#define LGAP_FRONTIER_BUFS 4
#endif
constexpr int kFrontierBufs = LGAP_FRONTIER_BUFS;  // depth-indexed row-index buffers
constexpr int kFrontierIdx = kFrontierBufs + 1;    // index buffers by id: depth buffers {0, 1, 3, ...}, bag 2
constexpr int kFrontierRoundCap = 64;  // rounds with their own expansion cap (later rounds: kmax)
constexpr int kFrontierMaxNodes = 4096;  // computed-node capacity of the select's LDS image
constexpr int kFrontierIcWords = 4;      // interaction-constraint sets on the frontier: 4 x 64

// Fixed-point exponent e of a sum over `rows` rows of values with max |v| = vmax and
// sum |v| <= vsum over ALL rows: the largest e with 2^e * min(rows * vmax, vsum) <= limit,
// so no partial sum over any subset of those rows can exceed `limit` in magnitude. The
// sum bound is what keeps heavy-tailed gradients (max|g| >> typical |g|) resolved: with
// rows * max alone, one outlier in 10M rows sets every row's quantum. 0 for a zero bound.
// (Shared by the kernels and the host test hooks, which must agree on the scale.)
__host__ __device__ inline int FixedPointExp(double limit, double rows, float vmax, float vsum) {
  double b = rows * static_cast<double>(vmax);
  if (static_cast<double>(vsum) < b) b = static_cast<double>(vsum);
  if (!(b > 0.0)) return 0;
  int e;
  (void)frexp(limit / b, &e);
  return e - 1;
}

// entries of the select's sort of the alive nodes: a power of two >= C (C <= kFrontierMaxNodes)
__host__ __device__ inline int FrontierSortCap(int C) {
  int p = 64;
  while (p < C) p <<= 1;
  return p;
}

// index-buffer id of depth buffer j (0..3)
__host__ __device__ inline int FrontierDepthBuf(int j) { return j < 2 ? j : j + 1; }

// node state bits (FArgs::nstate)
constexpr uint8_t kNodeExpanded = 1;   // children computed
constexpr uint8_t kNodeCommitted = 2;  // its split is part of the tree (replay)
constexpr uint8_t kNodeDead = 4;       // below an expansion the CEGB replay invalidated: never used
constexpr uint8_t kNodeStale = 0x40;   // (select-local) intermediate monotone: record scanned under looser bounds
constexpr uint8_t kNodeEligTmp = 0x20; // (select-local) eligible for expansion this round
constexpr uint8_t kNodeRescanTmp = 0x10;  // (select-local) re-scanned in the last round (new key)
constexpr uint8_t kNodeLocal = 0xF0;      // the select-local bits: never stored to FArgs::nstate
// stamp slots: kernel ids and the per-kernel slot count (slot 7: latest block exit)
constexpr int kFStampPart = 0, kFStampHist = 1, kFStampScan = 2, kFStampSel = 3, kFStampSlots = 8;

struct FNode {
  int buf, start, count;  // local rows: positions [start, start + count) of index buffer `buf`
  int gcount;             // global row count (data parallel: estimated from the split) / = count
  int depth, parent;
  int left;               // first child cid (right = left + 1), -1: not expanded
  int fidx;               // index of its forced split (FForced), -1: none
};

// Feature parallel: one rank's best candidate of one child (SplitInfo::BetterThan order).
struct FPairBest {
  SplitKey key;
  SplitInfo info;
};

// One forced split (forcedsplits_filename) in the host learner's application order
// (learner/forced_splits.h FlattenForced): inner feature, threshold bin, children indices.
struct FForced {
  int feature, threshold, left, right;
};

// One expansion (the split of node `parent`) of the current round.
struct FExp {
  int parent, left, depth;  // cids (right = left + 1); depth of the parent
  int tile0, ntiles;        // partition tiles [tile0, tile0 + ntiles)
  int src_buf, start, count;
  int dst_buf;
  // split predicate (the parent's SplitKey)
  int group, offset, num_bin, mfb, default_bin, missing, thr, default_left, is_cat;
  // written by the partition's post-split block
  int skip;                  // the children cannot split: no histogram / scan
  int smaller, larger;       // cids
  int h_buf, h_start, h_count;  // the smaller child's local rows
  int forced;                // the split is forced split `forced` (FForced index), -1: the node's best
  int feature;               // inner feature of the split (-1: the root pseudo-expansion)
  int last;                  // the tree's last split (the node the replay waits for, at num_leaves - 1
                             // leaves): its children are never scanned (as in the host's loop)
  int rescan;                // intermediate monotone: no split, node `smaller` is re-scanned from its slot
                             // under its tightened bounds (no tiles, no rows)
};

struct FState {
  int round;        // rounds run (including the root round)
  int k;            // expansions of the current round (rescans included)
  int kx;           // of which split a node (children cids [cid_next - 2 kx, cid_next)); the rest rescans
  int total_tiles;  // partition tiles of the current round
  int done;
  unsigned epoch;   // never reset: tags the partition's published tile counts
  int num_leaves, num_splits;
  int cid_next;
  int blocked;      // cid the replay waits for (-1: none)
  int spec;         // expansions started so far
  long long used_rows, waste_rows;  // (when done) rows partitioned by committed / uncommitted expansions
  int forced_next;  // next forced split to apply (-1: forced splits over or none)
  int byn;          // feature_fraction_bynode: masks drawn so far (the host's GetByNode calls)
  unsigned byn_rng; // by-node draws in the select (FArgs::byn_draw): the column sampler's LCG state
  int nsal;         // alive nodes in FArgs::salive (the last select's order; 0: none)
};

// Arguments of the frontier kernels (device pointers into the learner's buffers).
struct FArgs {
  const uint32_t* rowbins;
  const uint8_t* colbins;
  const float2* gh;  // class-major (cls from tp)
  int* idx[kFrontierIdx];
  int N, stride_dw, width, num_groups, TB, F, L, C, kmax;
  const int* gstart;
  const DevFeature* feat;
  const HistTile* tiles;
  int num_tiles;
  const uint8_t* used_bytree;
  const TreeParams* tp;
  // tree state
  FState* st;
  FNode* nodes;         // [C]
  FExp* exps;           // [kmax]
  uint32_t* exp_bits;   // [kmax][kMaxCatWords]: categorical left sets of the expansions
  double2* lsum;        // [C] (sum g, sum h)
  double* lout;         // [C] leaf outputs
  LeafBounds* bounds;   // [C]
  SplitKey* key;        // [C] best split (compact)
  SplitInfo* best;      // [C] best split (full)
  uint8_t* spl;         // [C][F] feature still splittable below this node
  unsigned long long* ic;        // [C][ic_words] interaction-constraint sets a node's path allows (null: none)
  const unsigned long long* ic_feat;  // [F][ic_words] the sets holding each feature
  int ic_words;                  // 64-set words (up to kFrontierIcWords: 256 sets)
  uint8_t* nstate;      // [C]
  int* leaf_cid;        // [L] committed leaf -> cid
  SplitRec* rec;        // [L - 1] committed splits in order
  LeafRange* range_out; // [L] final leaf ranges (written when done)
  // histograms
  double* slots;              // [C][2 TB] per-node histograms (stored bins, fp64)
  unsigned long long* acc;    // [kmax][2 TB] per-expansion fixed-point accumulators (zero between rounds)
  unsigned long long* hslab;  // [hist rows][hslab_stride] k_f_hist's per-block histograms (raw LDS words)
  size_t hslab_stride;        // words per slab row (TB, x2 for gpu_use_dp)
  long long* hmeta;           // [hist rows] MODE 0: the block's fixed-point exponents (bh << 32 | bg)
  int red_grid;               // k_f_reduce blocks
  // data-parallel owner-computes (reference data_parallel_tree_learner.cpp:284-297): the reduce
  // writes the round's accumulators as P per-rank chunks [xkb][own_w] (rank r's chunk = the bins of
  // the groups it owns, [own_b0[r], own_b0[r + 1])), a reduce-scatter sums each chunk into its
  // owner's acc_recv, the owner scans only its features and the per-child bests are all-gathered
  int own, own_P, own_rank, own_w;
  const int* own_b0;           // [P + 1]
  unsigned long long* acc_recv;  // [xkb][own_w] x (1 or 2 words)
  int xkb;                     // expansions the round's exchange covers (the chunk stride)
  const int* fown_list;        // owned features (scan items; null: every feature)
  int fown_n;
  const unsigned* ghmax;      // float bits of max|g|, max|h|, sum|g|, sum|h| over the root rows
  int sum_mult;               // ranks whose root rows the global sums span (row-sharded DP / voting), else 1
  int sum_bound;              // use the sum|value| bounds (LGAP_FIXED_SUMBOUND=0: max only, the round-3 scale)
  // forced splits: the list, and per node the forced split at its threshold (scan) and its
  // split predicate (for the expansion that applies it)
  const FForced* forced;
  int num_forced;
  SplitInfo* fbest;  // [C]
  SplitKey* fkey;    // [C]
  // quantized training (use_quantized_grad): per-row int8 levels, integer histograms
  const uint16_t* ghq;        // class-major: (g level int8) << 8 | (h level uint8)
  const unsigned* qmax;       // float bits of the quantizer's max|g|, max|h| (k_qmax)
  int quant;                  // 1: integer-level histograms (hist MODE 2)
  int qpack;                  // 1: one packed g32|h32 word per bin in the accumulator
  int qbins, qconst;          // num_grad_quant_bins, constant hessian
  int qsub;                   // > 0: 32-bit g16|h16 LDS bins (hist MODE 3), folded every qsub rows
  // candidates of the current round: [kmax][2][F]
  SplitKey* ckey;
  SplitInfo* cinfo;
  // partition look-back
  unsigned long long* tile_pub;
  unsigned* bar;
  int part_selfcount;  // test hook: every look-back counts its predecessor tiles itself (FTileCount)
  int hist_min_rows, hist_grid;
  int hist_threads;  // 512 or 1024 threads per histogram block
  int hist_il;       // bank-interleaved LDS histograms (tiles with pad = their largest group's bins)
  int scan_wave;     // k_f_scan_w (one wave per (expansion, feature)) instead of one block per item
  int scan_grid;     // cap of the block scan's grid (A/B knob LGAP_SCAN_GRID; 0: 4096)
  int hist_nib;       // rowbins / stride_dw / tiles describe 4-bit rows (8 groups per dword)
  int part_tile;  // rows per partition tile (256 x rows per thread)
  int max_depth, use_monotone;
  // intermediate monotone constraints (monotone_constraints_method=intermediate): the select keeps
  // each leaf's current bounds (cbnd), tightens them with the host's constraint walk as splits
  // commit, and re-scans leaves whose bounds moved past the ones their record was scanned with
  int mono_inter;
  LeafBounds* cbnd;  // [C] current bounds of the committed tree's leaves (by cid)
  int* salive;       // [C] the alive nodes by (gain desc, cid asc) as the last select ordered them
  double monotone_penalty;
  double cegb_split;  // cegb_tradeoff * cegb_penalty_split (per row of the node), 0: none
  // CEGB coupled feature penalties (cegb_penalty_feature_coupled) on the device, host
  // CegbPenalty semantics: the scan publishes RAW candidate gains (key.pad0 = monotone type)
  // and the select applies split / coupled / monotone penalties against the persistent
  // used-feature flags; a feature's first use in the replay refunds the other leaves' stored
  // candidates (leaf-index chain, as the host's per-leaf table) and invalidates speculation
  const double* cegb_coupled;  // [F] tradeoff x coupled penalty per inner feature, null: off
  double cegb_tradeoff;
  uint8_t* cegb_used;          // [F] feature used by a split (persists across trees)
  unsigned* cegb_epoch;        // [1] first-use events so far
  SplitKey* nkey;              // [C][F] every computed node's raw per-feature candidates
  SplitInfo* ninfo;            // [C][F]
  int* nuep;                   // [C] cegb_epoch its best was computed at
  int cegb_raw;                // 1: scans publish raw gains, the select applies the CEGB penalties
  // CEGB lazy per-row penalties (cegb_penalty_feature_lazy): a node's cost for feature f is
  // pen_f x its rows not yet marked for f (marks of earlier trees; features on the node's own
  // path count zero: the host marks a split leaf's rows for its feature as it splits)
  const double* cegb_lazy;     // [F] tradeoff x lazy penalty per inner feature, null: off
  uint32_t* lazy_bits;         // [N][lazy_words] per-row marks (features used on the row's path)
  int lazy_words;
  int* lazy_acc;               // [kmax][F] the round's smaller-child unmarked counts (zero between rounds)
  int* nlazy;                  // [C][F] unmarked counts per node
  uint32_t* npath;             // [C][lazy_words] features on the node's path
  int max_bin, cat_p2;
  int use_dp;       // gpu_use_dp: 64-bit LDS accumulators
  int spec_cap;     // speculative expansions per round beyond the budget (policy knob)
  int policy;       // 1: budget by global gain rank (default), 0: budget minus uncommitted expansions
  int distributed;  // children counts from the split record (global) instead of the partition
  const int* kcap;  // [kFrontierRoundCap] per-round expansion caps (data-parallel: the all-reduce sizes), or null
  int* kused;       // [kFrontierRoundCap] expansions each round actually took (host feedback), or null
  unsigned long long* stamps;  // diagnostics (LGAP_FSTAMPS=1): [round & 255][kernel 0..3][8] wall clock
  // expansion range [e_lo, e_hi) a k_f_hist / k_f_scan launch covers (data-parallel pipeline:
  // the first half's all-reduce runs on the comm stream while the second half's histograms
  // build); 0 / kFrontierKmax: the whole round
  int e_lo, e_hi;
  // Voting parallel (PV-Tree) on the frontier (k_f_scan is then the LOCAL pass): local leaf
  // statistics and min_data / min_hessian divided by the rank count, local top-k votes per
  // child, the elected features' fixed-point rows summed over ranks, a GLOBAL pass over them.
  // Reference: voting_parallel_tree_learner.cpp:243-399.
  int voting;
  int vote_k, vote_P, vote_rank;
  const SplitParams* sp_local;  // voting's local pass: min_data / min_hessian divided by the ranks (device memory)
  double2* lsum_loc;          // [C] local (sum g, sum h) of every computed node
  unsigned long long* ltot;   // [kmax][2] the round's smaller children's local totals (global fixed-point scale)
  VoteRec* vrec;              // [P][kmax][2][K] local top-k records, all-gathered
  int* velect;                // [kmax][2][K + 1] elected count, elected features ascending
  unsigned long long* vrows;  // [kmax][2][K][2 max_bin] elected features' local fixed-point rows, summed in place
  // Feature parallel on the frontier: every rank holds all rows and grows the same partition;
  // k_f_scan scans the features this rank owns (fowned), each child's best is all-gathered and
  // the best over ranks becomes the child's candidate. Reference: feature_parallel_tree_learner.cpp:23-80.
  const uint8_t* fowned;  // [F] 1: this rank scans the feature (null: every feature)
  // feature_fraction_bynode: the tree's by-node masks [2 L][F] in the host's draw order (the
  // root's, then smaller / larger child of every split whose children are scanned). Candidates
  // stay raw per node (cegb_raw); a node's mask is known once its parent commits, so the
  // replay scores the children then, and only leaves of the committed tree are expanded.
  const uint8_t* bynode;
  // by-node sampling under interaction constraints: a node's pool (the by-tree features its
  // constraints allow) depends on its path, so the masks cannot be drawn ahead. The select draws
  // rows 1.. itself when a split commits (smaller child first), Random::Sample over the pool with
  // the column sampler's LCG (FState::byn_rng; the host draws the root's row 0 and takes the
  // final state back), into byn_draw (== bynode). byn_mode[N]: Sample's branch for a pool of N
  // (0 none, 1 all, 2 Bernoulli scan, 3 Floyd; host-computed: its log2 test stays the host's).
  uint8_t* byn_draw;
  const uint8_t* byn_mode;
  int byn_cnt;    // GetCnt(by-tree feature count, feature_fraction_bynode)
  int byn_reset;  // by-tree sampling on: the pool is filtered by used_bytree
  // extra_trees: per-feature random streams (Random(extra_seed + f), persistent across trees;
  // null: off). Draws follow the host's order (each scanned node: smaller child, then larger),
  // which the frontier keeps by expanding only the node the replay is blocked on: at its scan
  // every earlier split of the sequential order is committed.
  unsigned* xrng;
  struct FPairBest* fpb;  // [P][kmax][2] per-child best of each rank, all-gathered
  SplitParams sp;
  // xGMI in-kernel exchange of the distributed frontier (owner-computes data parallel and feature
  // parallel; device_learner.hip SetupFrontierXgmi). Every rank holds one uncached exchange buffer
  // at identical offsets, IPC-mapped by every peer: k_f_reduce adds each histogram bin straight into
  // its OWNER's receive chunk (64-bit integer atomics over xGMI: exact, order free), k_f_pair_best
  // stores this rank's per-child bests into every peer's record table, and the last block of each
  // producing launch tags flag[kind][this rank] in every peer, then waits for all P tags of its own
  // (bounded: bar[3]). The consumer is the next kernel on the stream: no collective call, host
  // round trip or extra launch per round, and a tree replays as one hipGraph. Voting parallel: k_f_vote
// stores its top-k records into every rank's table, k_f_elect adds the elected features' local rows
// into every rank's row block (the all-gather and the exact all-reduce of the collectives path).
  int xg;                        // 1: in-kernel exchange (xc valid)
  unsigned xsession;             // high word of every tag (0: the set-up self-test)
  const struct FXConf* xc;       // the transport's per-learner constants (device memory)
};

// The xGMI transport's per-learner constants, in device memory (FArgs::xc): kept out of the kernel
// arguments, which every frontier launch of a round carries (FArgs stays under 1 KiB: measured
// ~0.5 us more per launch with the peers' pointers inline).
struct FXConf {
  char* peer[kMaxXRanks];        // rank q's exchange buffer in this process's address space
  size_t o_recv, o_fpb, o_root, o_flag;  // byte offsets inside every rank's buffer
  size_t o_vrec, o_vrows;        // voting: the top-k records [P][2 kmax][K], the elected rows (summed)
  unsigned* ep;                  // [1] rounds exchanged so far: a round's tag is (xsession, *ep + 1)
  unsigned* cnt;                 // [kFXKinds] block arrivals of the current producing launch
  unsigned long long timeout;    // wall-clock ticks (100 MHz) a wait may spin before it gives up
  int P, rank;
  int fault;                     // test hook (LGAP_FAULT_INJECT=xgmi): this rank never signals
  int pad;
};

// exchange kinds of the frontier's xGMI transport (flag rows of the exchange buffer)
constexpr int kFXHist = 0, kFXCand = 1, kFXRoot = 2, kFXVote = 3, kFXVRows = 4, kFXTest = 5, kFXKinds = 6;
// root exchange record: (sum g, sum h) and the four gradient bounds of k_f_init_root (float bits)
struct FXRoot {
  double g, h;
  unsigned m[4];
};

// Results of a replay, written by k_f_results straight into coherent pinned host memory (one
// small kernel instead of five D2H copies, each ~19 us apart on the copy path): the header,
// then (once the tree is done) SplitRec[L - 1] at FrontierResultRecOffset() and LeafRange[L]
// after them.
struct FResultHdr {
  FState st;
  unsigned bar[4];
  double lout0;
  int kused[kFrontierRoundCap];
};
__host__ __device__ inline size_t FrontierResultRecOffset() { return (sizeof(FResultHdr) + 15) & ~size_t(15); }
__host__ __device__ inline size_t FrontierResultRangeOffset(int L) {
  return FrontierResultRecOffset() + ((sizeof(SplitRec) * static_cast<size_t>(L > 1 ? L - 1 : 1) + 15) & ~size_t(15));
}
inline size_t FrontierResultBytes(int L) { return FrontierResultRangeOffset(L) + sizeof(LeafRange) * static_cast<size_t>(L); }

// launchers (frontier_kernels.hip)
void LaunchFrontierResults(const FArgs& a, void* host_out, hipStream_t s);
void LaunchFrontierInit(const FArgs& a, hipStream_t s);
// k_f_init + the fold of seq::k_root_sums' per-block partials (k_root_final's order) in one launch
void LaunchFrontierInitRoot(const FArgs& a, const double* root_part, int nblocks, unsigned* ghmax, hipStream_t s);
void LaunchFrontierHist(const FArgs& a, size_t lds_bytes, hipStream_t s);  // k_f_hist + k_f_reduce
int FrontierHistRows(int hist_grid, int kmax);  // k_f_hist's grid.x (partial slab rows)
void LaunchFrontierScan(const FArgs& a, size_t lds_bytes, hipStream_t s);

// Wave-per-item scan (k_f_scan_w, wide data): per wave the two fp64 (g, h) histograms of the
// widest feature and one categorical sort slot (index, ctr); four waves per block.
constexpr int kFScanWaves = 4;
__host__ __device__ inline size_t FrontierScanWaveBytes(int max_bin, int cat_p2) {
  const size_t b = static_cast<size_t>(max_bin) * 4 * sizeof(double) + static_cast<size_t>((cat_p2 + 1) & ~1) * sizeof(int) +
                   static_cast<size_t>(cat_p2) * sizeof(double);
  return (b + 15) & ~static_cast<size_t>(15);
}
void LaunchFrontierSelect(const FArgs& a, hipStream_t s);
// extra LDS of the intermediate-monotone select (after FrontierSelectLds): per-leaf current and
// scan bounds, per-node thresholds, the committed node's ancestor levels, per-feature monotone
// types
__host__ __device__ inline size_t FrontierSelectMonoLds(int C, int L, int F) {
  return 16 + static_cast<size_t>(L) * (2 * 16 + 3 * sizeof(int) + 1) + static_cast<size_t>(C) * sizeof(int) +
         static_cast<size_t>(F) + 16;
}
// CEGB lazy penalties: unmarked-row counts of the round's smaller children; after a tree, the
// final leaves' rows marked for the features on their paths
void LaunchFrontierLazyCounts(const FArgs& a, hipStream_t s);
void LaunchFrontierLazyMark(const FArgs& a, hipStream_t s);
void LaunchFrontierPartition(const FArgs& a, int iters, int grid, hipStream_t s);  // one block per tile
int FrontierPartitionBlocksPerCU(int iters);
// voting parallel: local top-k per child (after the local-pass k_f_scan), election and
// packing of the elected features' local rows (after the vote all-gather), global pass over
// the summed rows (after their all-reduce)
void LaunchFrontierVote(const FArgs& a, hipStream_t s);
void LaunchFrontierElect(const FArgs& a, hipStream_t s);
void LaunchFrontierVoteScan(const FArgs& a, size_t lds_bytes, hipStream_t s);
// feature parallel / owner-computes data parallel: this rank's per-child best -> fpb[rank] (before
// the all-gather; k_f_select's phase A takes the best over the ranks after it)
void LaunchFrontierPairBest(const FArgs& a, hipStream_t s);
// xGMI transport: the root sums / gradient bounds exchanged and folded in rank order (replaces the
// per-tree all-reduces), and the set-up self-test (round r: every rank adds a known pattern into
// every peer's receive chunk, then checks and clears its own; mismatches counted into err)
void LaunchFrontierXRoot(const FArgs& a, unsigned* ghmax, hipStream_t s);
void LaunchFrontierXSelfTest(const FArgs& a, int round, int nvals, unsigned* err, hipStream_t s);
// one-time kernel attributes (dynamic LDS above 64 KiB)
void FrontierSetLds(size_t hist_lds, size_t scan_lds, bool use_dp, int width);
// dynamic LDS of k_f_select (CEGB coupled penalties add F bytes of used flags after it)
__host__ __device__ inline size_t FrontierSelectLds(int C, int L) {
  return static_cast<size_t>(C) * (sizeof(double) + 6 * sizeof(int) + 1) + 64 +
         static_cast<size_t>(L) * (3 * sizeof(int) + sizeof(double) + sizeof(int)) + 64 +
         static_cast<size_t>(FrontierSortCap(C)) * (sizeof(double) + sizeof(int));
}


}  // namespace device
}  // namespace lgap
