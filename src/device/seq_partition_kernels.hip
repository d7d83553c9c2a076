// Sequential chain: best-leaf select, stable partition (two-kernel and fused decoupled
// look-back), post-split bookkeeping, leaf-value adds, score-update traversal and the
// row -> column transpose (declarations: seq_kernels.h).
#include "device/seq_kernels.h"

namespace lgap {
namespace device {
namespace seq {

__device__ __forceinline__ void CopySplitInfoBlock(SplitInfo* dst, const SplitInfo* src) {
  constexpr int kWords = static_cast<int>(sizeof(SplitInfo) / 4);
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
  uint32_t* d = reinterpret_cast<uint32_t*>(dst);
  for (int i = threadIdx.x; i < kWords; i += blockDim.x) d[i] = s[i];
}

// ---------------------------------------------------------------------------
// best-leaf selection, replicated in every block of k_part_count

__device__ __forceinline__ bool CandBetter(double ga, int fa, int la, double gb, int fb, int lb) {
  if (ga != gb) return ga > gb;
  if (fa != fb) return fa < fb;
  return la < lb;
}

struct SelState {
  int done;       // no further split
  int leaf;       // leaf to split
  int sel;        // winner source: 0/1 = candidate table row of the smaller/larger child, -1 = best[leaf]
  int feature;
  int new_best[2];  // candidate-table position of the smaller/larger child's best (-1: none)
};

// ---------------------------------------------------------------------------
// stable partition of the split leaf's row indices

__device__ void FillSplitDesc(const Args& a, const SplitInfo& s, SplitDesc* d) {
  const DevFeature fi = a.feat[s.feature];
  d->group = fi.group;
  d->offset = fi.offset;
  d->num_bin = fi.num_bin;
  d->mfb = fi.mfb;
  d->default_bin = fi.default_bin;
  d->missing = fi.missing;
  d->thr = static_cast<int>(s.threshold);
  d->default_left = s.default_left;
  d->is_cat = fi.bin_type != 0;
  for (int w = 0; w < kMaxCatWords; ++w) d->bits[w] = d->is_cat ? s.cat_bitset[w] : 0u;
}

__device__ __forceinline__ void WaveArgBest4(double* g, int* f, int* l, int* o) {
  const int src = WaveArgBestLane(*g, *f, *l);
  *g = ReadLane(*g, src);
  *f = ReadLane(*f, src);
  *l = ReadLane(*l, src);
  *o = ReadLane(*o, src);
}

struct SelOut {
  SelState st;
  SplitDesc d;
  LeafRange pr;
  SplitKey key[2];  // the two children's winning keys (persisted by block 0)
};

__device__ void SelectFromKeys(const Args& a, const Ctl& c, SelOut* so) {
  constexpr int kW = kPartThreads / 64;
  constexpr int kNone = 0x7fffffff;
  __shared__ double s_g[3][kW];
  __shared__ int s_f[3][kW], s_l[3][kW], s_o[3][kW];
  __shared__ int s_owner[3], s_win_cat;
  __shared__ LeafRange s_rng[kPartThreads];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  double g3[3] = {kMinScore, kMinScore, kMinScore};
  int f3[3] = {kNone, kNone, kNone};
  int l3[3] = {0, 0, kNone};
  SplitKey k3_0, k3_1, k3_2;  // (named: a runtime-indexed array would live in scratch)
  if (!c.skip) {
    // the two children's candidates: every position of the table (all ranks' blocks)
    const int np = a.cand_rows * a.Fmax;
#pragma unroll
    for (int sel = 0; sel < 2; ++sel) {
      const int leaf = sel ? c.larger : c.smaller;
      if (leaf < 0) continue;
      for (int p = t; p < np; p += blockDim.x) {
        const int r = p / a.Fmax;
        const SplitKey k = *CandKey(a, r, sel, p - r * a.Fmax);
        if (k.feature >= 0 && CandBetter(k.gain, k.feature, 0, g3[sel], f3[sel], 0)) {
          g3[sel] = k.gain;
          f3[sel] = k.feature;
          if (sel == 0) k3_0 = k;
          else k3_1 = k;
        }
      }
    }
  }
  for (int l = t; l < c.num_leaves; l += blockDim.x) {
    if (l == c.smaller || l == c.larger) continue;
    const SplitKey k = a.leaf_key[l];
    const double g = k.feature < 0 ? kMinScore : k.gain;
    const int f = k.feature < 0 ? kNone : k.feature;
    if (CandBetter(g, f, l, g3[2], f3[2], l3[2])) {
      g3[2] = g;
      f3[2] = f;
      l3[2] = l;
      k3_2 = k;
    }
  }
  if (t <= c.num_leaves && t < kPartThreads) s_rng[t] = a.range[t];
  Stamp(a, 0, 4);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    int o = t;
    WaveArgBest4(&g3[k], &f3[k], &l3[k], &o);
    if (lane == 0) {
      s_g[k][w] = g3[k];
      s_f[k][w] = f3[k];
      s_l[k][w] = l3[k];
      s_o[k][w] = o;
    }
  }
  __syncthreads();
  Stamp(a, 0, 5);
  if (t == 0) {
    for (int k = 0; k < 3; ++k) {
      for (int i = 1; i < kW; ++i) {
        if (CandBetter(s_g[k][i], s_f[k][i], s_l[k][i], s_g[k][0], s_f[k][0], s_l[k][0])) {
          s_g[k][0] = s_g[k][i];
          s_f[k][0] = s_f[k][i];
          s_l[k][0] = s_l[k][i];
          s_o[k][0] = s_o[k][i];
        }
      }
      s_owner[k] = s_f[k][0] == kNone ? -1 : s_o[k][0];
    }
    SelState& st = so->st;
    st.new_best[0] = -1;  // positions: filled in by the owning threads below
    st.new_best[1] = -1;
    double bg = s_g[2][0];
    int bf = s_f[2][0], bl = s_l[2][0], cat = 2;
    for (int sel = 0; sel < 2; ++sel) {
      const int leaf = sel ? c.larger : c.smaller;
      if (leaf < 0 || s_f[sel][0] == kNone) continue;
      if (CandBetter(s_g[sel][0], s_f[sel][0], leaf, bg, bf, bl)) {
        bg = s_g[sel][0];
        bf = s_f[sel][0];
        bl = leaf;
        cat = sel;
      }
    }
    st.leaf = bl;
    st.feature = bf;
    st.done = (bl == kNone || bf == kNone || !(bg > 0.0)) ? 1 : 0;
    st.sel = cat == 2 ? -1 : cat;
    s_win_cat = st.done ? -1 : cat;
  }
  __syncthreads();
  if (t == s_owner[0]) {
    so->key[0] = k3_0;
    so->st.new_best[0] = k3_0.pos;
  }
  if (t == s_owner[1]) {
    so->key[1] = k3_1;
    so->st.new_best[1] = k3_1.pos;
  }
  const int wc = s_win_cat;
  if (wc >= 0 && t == s_owner[wc]) {
    const SplitKey k = wc == 0 ? k3_0 : (wc == 1 ? k3_1 : k3_2);
    SplitDesc& d = so->d;
    d.group = k.group;
    d.offset = k.offset;
    d.num_bin = k.num_bin;
    d.mfb = k.mfb;
    d.default_bin = k.default_bin;
    d.missing = k.missing;
    d.thr = static_cast<int>(k.threshold);
    d.default_left = k.default_left;
    d.is_cat = k.is_cat;
    if (k.is_cat) {
      const SplitInfo* win = wc < 2 ? CandInfoPos(a, wc, k.pos) : &a.best[so->st.leaf];
      for (int i = 0; i < kMaxCatWords; ++i) d.bits[i] = win->cat_bitset[i];
    }
    const int leaf = so->st.leaf;
    so->pr = leaf < kPartThreads ? s_rng[leaf] : a.range[leaf];
  }
  Stamp(a, 0, 6);
  __syncthreads();
}


// Block 0 of the partition: persist the two children's bests (full record + compact
// key) for later selects, and the `done` decision in both control buffers.
__device__ void PersistChildBests(const Args& a, const Ctl& c, const SelOut& so) {
  const SelState& st = so.st;
  if (c.smaller >= 0 && st.new_best[0] >= 0) CopySplitInfoBlock(&a.best[c.smaller], CandInfoPos(a, 0, st.new_best[0]));
  if (c.larger >= 0 && st.new_best[1] >= 0) CopySplitInfoBlock(&a.best[c.larger], CandInfoPos(a, 1, st.new_best[1]));
  if (threadIdx.x == 0) {
    if (c.smaller >= 0) {
      if (st.new_best[0] >= 0) {
        a.leaf_key[c.smaller] = so.key[0];
      } else {
        a.best[c.smaller].Reset();
        a.leaf_key[c.smaller].feature = -1;
        a.leaf_key[c.smaller].gain = kMinScore;
      }
    }
    if (c.larger >= 0) {
      if (st.new_best[1] >= 0) {
        a.leaf_key[c.larger] = so.key[1];
      } else {
        a.best[c.larger].Reset();
        a.leaf_key[c.larger].feature = -1;
        a.leaf_key[c.larger].gain = kMinScore;
      }
    }
    if (st.done) {
      // both control buffers: later launches read either
      a.ctl->done = 1;
      a.ctl_next->done = 1;
    }
  }
}

// Select the leaf to split (replicated), persist the decision (block 0), then
// count the rows going left per 4096-row tile of the parent range.
__global__ __launch_bounds__(kPartThreads) void k_part_count(Args a) {
  __shared__ SelOut so;
  __shared__ int sh[8];
  Ctl* cp = a.ctl;
  const Ctl c = *cp;
  if (c.done) return;
  // no leaf has more tiles than this: surplus blocks have nothing to count
  if (blockIdx.x > 0 && static_cast<int>(blockIdx.x) >= (c.max_count + kTileRows - 1) / kTileRows) return;
  Stamp(a, 0, 0);
  SelectFromKeys(a, c, &so);
  Stamp(a, 0, 1);
  const SelState& st = so.st;
  if (blockIdx.x == 0) PersistChildBests(a, c, so);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (!c.skip) cp->scan_round = c.scan_round + 1;
    if (!st.done) {
      const LeafRange pr = so.pr;
      cp->split_leaf = st.leaf;
      cp->new_leaf = c.num_leaves;
      cp->parent_buf = pr.buf;
      cp->parent_start = pr.start;
      cp->parent_count = pr.count;
      cp->target_buf = pr.buf == 0 ? 1 : 0;
    }
  }
  if (st.done) return;
  const SplitDesc& d = so.d;
  const LeafRange pr = so.pr;
  Stamp(a, 0, 2);
  const int ntiles = (pr.count + kTileRows - 1) / kTileRows;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // all 16 index loads in flight, then all 16 split-column loads
    int rows[kPartIters];
    const int pos0 = tile * kTileRows + threadIdx.x;
#pragma unroll
    for (int k = 0; k < kPartIters; ++k) {
      const int pos = pos0 + k * kPartThreads;
      rows[k] = pos < pr.count ? RowAt(a, pr.buf, pr.start + pos) : -1;
    }
    uint32_t gb[kPartIters];
#pragma unroll
    for (int k = 0; k < kPartIters; ++k) gb[k] = rows[k] >= 0 ? ColBin(a, d.group, rows[k]) : 0u;
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < kPartIters; ++k) cnt += (rows[k] >= 0 && GoLeft(d, gb[k])) ? 1 : 0;
    cnt = BlockSumInt(cnt, sh);
    if (threadIdx.x == 0) a.tile_cnt[tile] = cnt;
  }
  Stamp(a, 0, 3);
}

// Post-split bookkeeping (BeforeFindBestSplit of the two children); run by
// block 0 of k_part_scatter after its own tiles. Touches only state that no
// other k_part_scatter block reads. All loads are issued before any store.
// `win` is the applied split: best[split_leaf] in the two-kernel path, or the
// record the fused kernel selected from (visible to every block: written by an
// earlier kernel, unlike best[] entries persisted by block 0 in the same launch).
__device__ void PostSplit(const Args& a, const Ctl& c, int left_count, const SplitInfo* win) {
  __shared__ int s_skip, s_from, s_to;
  const int l = c.split_leaf, r = c.new_leaf;
  if (threadIdx.x == 0) {
    const SplitInfo& bi = *win;
    const double lsg = bi.left_sum_gradient, lsh = bi.left_sum_hessian;
    const double rsg = bi.right_sum_gradient, rsh = bi.right_sum_hessian;
    const double lo = bi.left_output, ro = bi.right_output;
    const int ilc = bi.left_count, irc = bi.right_count;
    const int8_t mono = bi.monotone_type;
    const int16_t ncat = bi.num_cat_threshold;
    if (a.ic_leaf) {
      const unsigned long long m = a.ic_leaf[l] & a.ic_feat[bi.feature];
      a.ic_leaf[l] = m;
      a.ic_leaf[r] = m;
    }
    const int dep = a.depth[l] + 1;
    LeafBounds bl = a.bounds[l];
    const int ps = a.slot[l];
    // ---- stores
    const int lc = left_count, rc = c.parent_count - lc;
    LeafRange rl, rr;
    rl.buf = rr.buf = c.target_buf;
    rl.start = c.parent_start;
    rl.count = lc;
    rr.start = c.parent_start + lc;
    rr.count = rc;
    rl.pad = rr.pad = 0;
    a.range[l] = rl;
    a.range[r] = rr;
    const int glc = a.distributed ? ilc : lc;
    const int grc = a.distributed ? irc : rc;
    SplitRec& rec = a.rec[c.num_splits];
    rec.leaf = l;
    rec.left_count = glc;
    rec.right_count = grc;
    rec.pad = 0;
    a.lsum[l] = make_double2(lsg, lsh);
    a.lsum[r] = make_double2(rsg, rsh);
    a.lout[l] = lo;
    a.lout[r] = ro;
    a.gcount[l] = glc;
    a.gcount[r] = grc;
    a.depth[l] = dep;
    a.depth[r] = dep;
    LeafBounds br = bl;
    if (a.use_monotone && ncat == 0) {
      const double mid = (lo + ro) / 2.0f;
      if (mono < 0) {
        bl.min = fmax(bl.min, mid);
        br.max = fmin(br.max, mid);
      } else if (mono > 0) {
        bl.max = fmin(bl.max, mid);
        br.min = fmax(br.min, mid);
      }
    }
    a.bounds[l] = bl;
    a.bounds[r] = br;
    const int smaller = glc < grc ? l : r;
    const int larger = glc < grc ? r : l;
    const int md = a.sp.min_data_in_leaf;
    const bool skip = (a.max_depth > 0 && dep >= a.max_depth) || (grc < md * 2 && glc < md * 2);
    Ctl nc = c;
    if (a.lsum_loc) {
      // voting: the split leaf's local sums, for the larger child's local pass
      const double2 pl = a.lsum_loc[l];
      nc.plg = pl.x;
      nc.plh = pl.y;
    }
    nc.num_splits = c.num_splits + 1;
    nc.num_leaves = c.num_leaves + 1;
    nc.left_count = lc;
    nc.smaller = smaller;
    nc.larger = larger;
    nc.skip = skip ? 1 : 0;
    nc.epoch = c.epoch + 1u;
    int to = -1;
    if (!skip) {
      if (larger == r) {
        a.slot[r] = ps;
        a.slot[l] = r;
        to = r;
      } else {
        a.slot[r] = r;
        to = r;
      }
    }
    *a.ctl_next = nc;
    s_from = ps;
    s_to = to;
    s_skip = skip ? 1 : 0;
  }
  // the split record (dword-parallel copy of the winning SplitInfo)
  CopySplitInfoBlock(&a.rec[c.num_splits].info, win);
  // largest leaf after this split (grid bound of the next partition kernels)
  {
    __shared__ int s_mx[kPartThreads / 64];
    int mx = 0;
    for (int q = threadIdx.x; q <= c.num_leaves; q += blockDim.x) {
      int cnt;
      if (q == l) cnt = left_count;
      else if (q == r) cnt = c.parent_count - left_count;
      else cnt = a.range[q].count;
      mx = max(mx, cnt);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, kWave));
    if ((threadIdx.x & 63) == 0) s_mx[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int i = 1; i < static_cast<int>(blockDim.x >> 6); ++i) mx = max(mx, s_mx[i]);
      a.ctl_next->max_count = mx;
    }
  }
  __syncthreads();
  if (!s_skip) {
    const uint8_t* src = a.splittable + static_cast<size_t>(s_from) * a.F;
    uint8_t* dst = a.splittable + static_cast<size_t>(s_to) * a.F;
    for (int f = threadIdx.x; f < a.F; f += blockDim.x) dst[f] = src[f];
  }
}

// Scatter rows into the target index buffer (stable: lefts in order, then
// rights in order). Each block derives its tiles' offsets from the tile counts
// itself; block 0 finishes with the post-split bookkeeping.
__global__ __launch_bounds__(kPartThreads) void k_part_scatter(Args a) {
  __shared__ SplitDesc d;
  __shared__ int s_wl[kPartIters][kPartThreads / 64];
  __shared__ int s_wv[kPartIters][kPartThreads / 64];
  __shared__ int sh[8];
  const Ctl* cp = a.ctl;
  const Ctl c = *cp;
  if (c.done) return;
  const int pbuf = c.parent_buf, pstart = c.parent_start, pcount = c.parent_count;
  const int ntiles = (pcount + kTileRows - 1) / kTileRows;
  // the post-split bookkeeping runs on the first block without tiles (in parallel
  // with the scatter), or after block 0's tiles when every block has tiles
  const int post_block = (a.fuse_post == 2 && ntiles < static_cast<int>(gridDim.x)) ? ntiles : 0;
  const int bid = static_cast<int>(blockIdx.x);
  if (bid > 0 && bid >= ntiles && bid != post_block) return;
  int* out = a.idx[c.target_buf] + pstart;
  Stamp(a, 1, 0);
  if (threadIdx.x == 0 && bid < ntiles) FillSplitDesc(a, a.best[c.split_leaf], &d);
  int nl = 0;
  for (int i = threadIdx.x; i < ntiles; i += blockDim.x) nl += a.tile_cnt[i];
  const int nl_total = BlockSumInt(nl, sh);
  Stamp(a, 1, 1);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    int pre = 0;
    for (int i = threadIdx.x; i < tile; i += blockDim.x) pre += a.tile_cnt[i];
    int lbase = BlockSumInt(pre, sh);
    int rbase = tile * kTileRows - lbase;
    int rows[kPartIters];
    const int pos0 = tile * kTileRows + threadIdx.x;
#pragma unroll
    for (int k = 0; k < kPartIters; ++k) {
      const int pos = pos0 + k * kPartThreads;
      rows[k] = pos < pcount ? RowAt(a, pbuf, pstart + pos) : -1;
    }
    uint32_t gb[kPartIters];
#pragma unroll
    for (int k = 0; k < kPartIters; ++k) gb[k] = rows[k] >= 0 ? ColBin(a, d.group, rows[k]) : 0u;
#pragma unroll
    for (int k = 0; k < kPartIters; ++k) {
      const bool valid = rows[k] >= 0;
      const bool left = valid && GoLeft(d, gb[k]);
      const unsigned long long ml = __ballot(left);
      const unsigned long long mv = __ballot(valid);
      if (lane == 0) {
        s_wl[k][w] = __popcll(ml);
        s_wv[k][w] = __popcll(mv);
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPartIters; ++k) {
      const bool valid = rows[k] >= 0;
      const bool left = valid && GoLeft(d, gb[k]);
      const unsigned long long ml = __ballot(left);
      const unsigned long long mv = __ballot(valid);
      int pl = 0, pv = 0, tl = 0, tv = 0;
#pragma unroll
      for (int i = 0; i < kPartThreads / 64; ++i) {
        if (i < w) {
          pl += s_wl[k][i];
          pv += s_wv[k][i];
        }
        tl += s_wl[k][i];
        tv += s_wv[k][i];
      }
      if (valid) {
        const int rl = pl + __popcll(ml & lt_mask);
        const int rv = pv + __popcll(mv & lt_mask);
        if (left) out[lbase + rl] = rows[k];
        else out[nl_total + rbase + (rv - rl)] = rows[k];
      }
      lbase += tl;
      rbase += tv - tl;
    }
    __syncthreads();
  }
  Stamp(a, 1, 2);
  if (bid == post_block && a.fuse_post) PostSplit(a, c, nl_total, &a.best[c.split_leaf]);
  Stamp(a, 1, 3);
}

// ---------------------------------------------------------------------------
// Fused partition (select + count + scatter + post-split in ONE launch), with no
// grid barrier:
//  * select reads only compact SplitKeys (children's per-feature candidates, the
//    older leaves' bests) and the leaf ranges in one round of independent loads;
//    the winner's key is the partition predicate, no dependent descriptor loads;
//  * every block publishes its tiles' left counts as 64-bit {epoch, count}
//    granules (one agent-scope store each, no fences needed);
//  * a tile waits only for its PREDECESSORS' counts (decoupled look-back): lefts go
//    to [0, nl) in order, rights are placed from the END of the range in reverse
//    order, which needs the rights before the tile, not the global left total;
//  * a spare block (or block 0) gathers all counts for the total and runs the
//    post-split bookkeeping concurrently with the scatter.
// The control block it reads (a.ctl) is never written during the launch: the
// post-split state goes to a.ctl_next (double buffer), so no block can observe a
// half-updated split. Histograms are order independent (fixed point), so the
// reversed right child changes no result. Every wait is bounded: a timeout raises
// the sticky error flag bar[2] that the host checks after the tree.

__device__ __forceinline__ void PublishCount(unsigned long long* p, unsigned epoch, int cnt) {
  const unsigned long long v = (static_cast<unsigned long long>(epoch) << 32) | static_cast<unsigned>(cnt);
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// count of tile i of this split (bounded spin; on timeout raise the error flag and use 0)
__device__ __forceinline__ int AwaitCount(const Args& a, int i, unsigned epoch) {
  unsigned spins = 0;
  for (;;) {
    const unsigned long long v = __hip_atomic_load(&a.tile_pub[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (static_cast<unsigned>(v >> 32) == epoch) return static_cast<int>(static_cast<unsigned>(v));
    __builtin_amdgcn_s_sleep(1);
    if ((++spins & 1023u) == 0u &&
        (spins > (1u << 22) || __hip_atomic_load(&a.bar[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)) {
      __hip_atomic_store(&a.bar[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return 0;
    }
  }
}

// sum of the published counts of tiles [0, n)
__device__ int SumCounts(const Args& a, int n, unsigned epoch, int* sh) {
  int s = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += AwaitCount(a, i, epoch);
  return BlockSumInt(s, sh);
}

// ITERS rows per thread: tiles of 256 * ITERS rows. Smaller tiles spread a leaf over more
// blocks (more loads in flight, shorter look-back chains per block); A/B on MI355X:
// 10M rows 8 > 16 (+6%) and 4, 1.25M rows 4 > 8 > 16 (+18% over 16). See PartIters().
template <int ITERS>
__global__ __launch_bounds__(kPartThreads) void k_partition(Args a) {
  constexpr int kTile = kPartThreads * ITERS;
  __shared__ SelOut so;
  __shared__ int sh[8];
  __shared__ int s_wl[ITERS][kPartThreads / 64];
  __shared__ int s_wv[ITERS][kPartThreads / 64];
  const unsigned long long t_start = a.stamps ? wall_clock64() : 0ull;
  const Ctl c = *a.ctl;
  if (c.done) return;
  const int bid = static_cast<int>(blockIdx.x);
  // no leaf has more tiles than this; one block beyond may be the post-split block
  if (bid > (c.max_count + kTile - 1) / kTile) return;
  Stamp(a, 0, 0);
  SelectFromKeys(a, c, &so);
  Stamp(a, 0, 1);
  const SelState& st = so.st;
  if (bid == 0) PersistChildBests(a, c, so);
  if (st.done) return;
  const SplitInfo* win = st.sel >= 0 ? CandInfoPos(a, st.sel, st.new_best[st.sel]) : &a.best[st.leaf];
  const LeafRange pr = so.pr;
  const SplitDesc& d = so.d;
  const unsigned epoch = c.epoch;
  const int ntiles = (pr.count + kTile - 1) / kTile;
  const int participants = ntiles < static_cast<int>(gridDim.x) ? ntiles : static_cast<int>(gridDim.x);
  const bool has_post_block = participants < static_cast<int>(gridDim.x);
  const int post_block = has_post_block ? participants : 0;
  if (bid >= participants && bid != post_block) return;
  Stamp(a, 0, 2);
  const int pbuf = pr.buf, pstart = pr.start, pcount = pr.count;
  const int tbuf = pbuf == 0 ? 1 : 0;
  int* out = a.idx[tbuf] + pstart;
  // phase 1: count this block's tiles and publish them (the first tile's rows stay in registers)
  int rows0[ITERS];
  uint32_t gb0[ITERS];
  for (int tile = bid; tile < ntiles; tile += gridDim.x) {
    int rows[ITERS];
    const int pos0 = tile * kTile + threadIdx.x;
#pragma unroll
    for (int k = 0; k < ITERS; ++k) {
      const int pos = pos0 + k * kPartThreads;
      rows[k] = pos < pcount ? RowAt(a, pbuf, pstart + pos) : -1;
    }
    uint32_t gb[ITERS];
#pragma unroll
    for (int k = 0; k < ITERS; ++k) gb[k] = rows[k] >= 0 ? ColBin(a, d.group, rows[k]) : 0u;
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < ITERS; ++k) cnt += (rows[k] >= 0 && GoLeft(d, gb[k])) ? 1 : 0;
    cnt = BlockSumInt(cnt, sh);
    if (threadIdx.x == 0) PublishCount(&a.tile_pub[tile], epoch, cnt);
    if (tile == bid) {
#pragma unroll
      for (int k = 0; k < ITERS; ++k) {
        rows0[k] = rows[k];
        gb0[k] = gb[k];
      }
    }
  }
  Stamp(a, 0, 3);
  // the post-split block: total lefts from every tile, bookkeeping next to the scatter
  if (has_post_block && bid == post_block) {
    const int nl_total = SumCounts(a, ntiles, epoch, sh);
    const unsigned long long t_cnt = a.stamps ? wall_clock64() : 0ull;
    Ctl pc = c;
    pc.split_leaf = st.leaf;
    pc.new_leaf = c.num_leaves;
    pc.parent_buf = pbuf;
    pc.parent_start = pstart;
    pc.parent_count = pcount;
    pc.target_buf = tbuf;
    if (!c.skip) pc.scan_round = c.scan_round + 1;
    pc.hist_nb = 0;
    PostSplit(a, pc, nl_total, win);
    if (a.stamps) {
      StampAt(a, 4, c.num_splits, 0, t_start);
      StampAt(a, 4, c.num_splits, 1, t_cnt);
      StampAt(a, 4, c.num_splits, 2, wall_clock64());
    }
    return;
  }
  // phase 2: per tile, lefts before it (look-back) -> scatter
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int tile = bid; tile < ntiles; tile += gridDim.x) {
    int lbase = SumCounts(a, tile, epoch, sh);
    if (tile == bid) Stamp(a, 1, 0);
    int rbase = tile * kTile - lbase;  // rights before this tile
    int rows[ITERS];
    uint32_t gb[ITERS];
    if (tile == bid) {
#pragma unroll
      for (int k = 0; k < ITERS; ++k) {
        rows[k] = rows0[k];
        gb[k] = gb0[k];
      }
    } else {
      const int pos0 = tile * kTile + threadIdx.x;
#pragma unroll
      for (int k = 0; k < ITERS; ++k) {
        const int pos = pos0 + k * kPartThreads;
        rows[k] = pos < pcount ? RowAt(a, pbuf, pstart + pos) : -1;
      }
#pragma unroll
      for (int k = 0; k < ITERS; ++k) gb[k] = rows[k] >= 0 ? ColBin(a, d.group, rows[k]) : 0u;
    }
#pragma unroll
    for (int k = 0; k < ITERS; ++k) {
      const bool valid = rows[k] >= 0;
      const bool left = valid && GoLeft(d, gb[k]);
      const unsigned long long ml = __ballot(left);
      const unsigned long long mv = __ballot(valid);
      if (lane == 0) {
        s_wl[k][w] = __popcll(ml);
        s_wv[k][w] = __popcll(mv);
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < ITERS; ++k) {
      const bool valid = rows[k] >= 0;
      const bool left = valid && GoLeft(d, gb[k]);
      const unsigned long long ml = __ballot(left);
      const unsigned long long mv = __ballot(valid);
      int pl = 0, pv = 0, tl = 0, tv = 0;
#pragma unroll
      for (int i = 0; i < kPartThreads / 64; ++i) {
        if (i < w) {
          pl += s_wl[k][i];
          pv += s_wv[k][i];
        }
        tl += s_wl[k][i];
        tv += s_wv[k][i];
      }
      if (valid) {
        const int rl = pl + __popcll(ml & lt_mask);
        const int rv = pv + __popcll(mv & lt_mask);
        if (left) out[lbase + rl] = rows[k];
        else out[pcount - 1 - (rbase + (rv - rl))] = rows[k];  // rights fill the range from its end
      }
      lbase += tl;
      rbase += tv - tl;
    }
    __syncthreads();
  }
  Stamp(a, 1, 2);
  if (!has_post_block && bid == 0) {
    // every block has tiles: block 0 runs the post-split after its own
    const int nl_total = SumCounts(a, ntiles, epoch, sh);
    Ctl pc = c;
    pc.split_leaf = st.leaf;
    pc.new_leaf = c.num_leaves;
    pc.parent_buf = pbuf;
    pc.parent_start = pstart;
    pc.parent_count = pcount;
    pc.target_buf = tbuf;
    if (!c.skip) pc.scan_round = c.scan_round + 1;
    pc.hist_nb = 0;
    PostSplit(a, pc, nl_total, win);
  }
  if (a.stamps && threadIdx.x == 0) {
    atomicMax(&a.stamps[((static_cast<size_t>(0) * 256 + (c.num_splits & 255)) * 2) * 8 + 7], wall_clock64());
  }
}

__global__ __launch_bounds__(kPartThreads) void k_post(Args a) {
  __shared__ int sh[8];
  const Ctl c = *a.ctl;
  if (c.done) return;
  const int ntiles = (c.parent_count + kTileRows - 1) / kTileRows;
  int nl = 0;
  for (int i = threadIdx.x; i < ntiles; i += blockDim.x) nl += a.tile_cnt[i];
  PostSplit(a, c, BlockSumInt(nl, sh), &a.best[c.split_leaf]);
}

// ---------------------------------------------------------------------------
// score update: traverse one uploaded tree over the packed rows

// One row per thread. A block first stages its 256 contiguous packed rows in LDS
// with coalesced dword loads (rows are stride_dw dwords, not 16 B aligned), so
// the per-level bin reads of the traversal are LDS hits instead of dependent
// global loads; rows wider than kTraverseMaxDw read global memory directly.

__device__ __forceinline__ bool NodeGoLeft(const DevNode& nd, uint32_t gb, const uint32_t* __restrict__ cat_bits) {
  const uint32_t b = DecodeBin(nd.offset, nd.num_bin, nd.mfb, gb);
  if (nd.decision & 1) {
    const uint32_t wd = b >> 5;
    return static_cast<int>(wd) < nd.cat_nwords && ((cat_bits[nd.cat_begin + wd] >> (b & 31u)) & 1u);
  }
  if ((nd.missing == 1 && b == static_cast<uint32_t>(nd.default_bin)) ||
      (nd.missing == 2 && b == static_cast<uint32_t>(nd.num_bin - 1))) {
    return (nd.decision & 2) != 0;
  }
  return b <= static_cast<uint32_t>(nd.threshold);
}

__global__ __launch_bounds__(kTraverseThreads) void k_add_tree(const uint32_t* __restrict__ rowbins, int stride_dw,
                                                               int width, int N, const DevNode* __restrict__ nodes,
                                                               int num_nodes, const uint32_t* __restrict__ cat_bits,
                                                               const double* __restrict__ leaf_value,
                                                               double* __restrict__ score) {
  extern __shared__ uint32_t s_dyn[];
  DevNode* s_nodes = reinterpret_cast<DevNode*>(s_dyn);
  uint32_t* s_rows = s_dyn + num_nodes * (sizeof(DevNode) / 4);
  for (int i = threadIdx.x; i < num_nodes; i += blockDim.x) s_nodes[i] = nodes[i];
  const bool staged = stride_dw <= kTraverseMaxDw;
  for (long long base = static_cast<long long>(blockIdx.x) * kTraverseThreads; base < N;
       base += static_cast<long long>(gridDim.x) * kTraverseThreads) {
    const int rows = static_cast<int>(min(static_cast<long long>(kTraverseThreads), N - base));
    const int i = static_cast<int>(base) + threadIdx.x;
    const uint8_t* row;
    if (staged) {
      __syncthreads();  // previous chunk's readers are done (and the nodes are in place)
      const uint32_t* src = rowbins + base * stride_dw;
      const int ndw = rows * stride_dw;
      for (int k = threadIdx.x; k < ndw; k += kTraverseThreads) s_rows[k] = src[k];
      __syncthreads();
      row = reinterpret_cast<const uint8_t*>(s_rows + threadIdx.x * stride_dw);
    } else {
      if (base == static_cast<long long>(blockIdx.x) * kTraverseThreads) __syncthreads();
      row = reinterpret_cast<const uint8_t*>(rowbins + static_cast<size_t>(i) * stride_dw);
    }
    if (threadIdx.x >= rows) continue;
    int node = 0;
    while (node >= 0) {
      const DevNode& nd = s_nodes[node];
      const uint32_t gb = width == 1 ? row[nd.group] : reinterpret_cast<const uint16_t*>(row)[nd.group];
      node = NodeGoLeft(nd, gb, cat_bits) ? nd.left : nd.right;
    }
    score[i] += leaf_value[~node];
  }
}

// group-major copy of the packed rows: col[g * N + i] = group bin g of row i (coalesced writes;
// each row's dword run is read by consecutive groups' threads of other waves through L2)
template <typename T>
__global__ __launch_bounds__(256) void k_transpose_bins(const uint32_t* __restrict__ rowbins, int stride_dw, int N, int G,
                                                        uint8_t* __restrict__ colbins) {
  const long long total = static_cast<long long>(G) * N;
  for (long long idx = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; idx < total;
       idx += static_cast<long long>(gridDim.x) * blockDim.x) {
    const int g = static_cast<int>(idx / N);
    const int i = static_cast<int>(idx - static_cast<long long>(g) * N);
    const T* row = reinterpret_cast<const T*>(rowbins + static_cast<size_t>(i) * stride_dw);
    reinterpret_cast<T*>(colbins)[idx] = row[g];
  }
}

// ---------------------------------------------------------------------------


// instantiations launched by the DeviceTreeLearner
template __global__ void k_partition<4>(Args);
template __global__ void k_partition<8>(Args);
template __global__ void k_partition<16>(Args);
template __global__ void k_transpose_bins<uint8_t>(const uint32_t* __restrict__, int, int, int, uint8_t* __restrict__);
template __global__ void k_transpose_bins<uint16_t>(const uint32_t* __restrict__, int, int, int, uint8_t* __restrict__);

}  // namespace seq
}  // namespace device
}  // namespace lgap
