// Sequential chain: k_reduce_scan, the per-feature slab fold / owner-row sum and threshold
// scans (declarations: seq_kernels.h).
#include "device/seq_kernels.h"

namespace lgap {
namespace device {
namespace seq {

template <typename Acc, bool kGlobal>
__global__ __launch_bounds__(kScanThreads) void k_reduce_scan(Args a, int hist_grid) {
  extern __shared__ __align__(16) unsigned char smem_dyn[];
  // (kGlobal launches never split the fold: blockIdx.x is the feature slot)
  unsigned char* smem = kGlobal ? reinterpret_cast<unsigned char*>(a.scan_scratch) + blockIdx.x * a.scan_scratch_stride
                                : smem_dyn;
  const Ctl c = *a.ctl;
  if (c.done || c.skip) return;
  const int C = a.fold_chunks;
  int j = blockIdx.x, ch = 0;
  if (C > 1) {
    // the C chunk blocks of a feature take consecutive places in XCD order (blocks b and b + 8
    // usually share an XCD, so the last arriver reads its partners' runs from its own L2;
    // speed only): the grid is padded to a multiple of 8
    const int q = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    j = q / C;
    ch = q - j * C;
    if (j >= a.fold_feats) return;
  }
  const int f = a.own_feat ? a.own_feat[j] : j;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  Stamp(a, 3, 0);
  __shared__ int s_skip_both, s_rand[2];
  __shared__ double s_sum[2][2];
  __shared__ __align__(8) unsigned char s_out_raw[2 * sizeof(SplitInfo)];
  __shared__ SplitKey s_key[2];
  SplitInfo* s_out = reinterpret_cast<SplitInfo*>(s_out_raw);
  if (t < 2) {
    s_out[t].Reset();
    SplitKey k;
    k.gain = kMinScore;
    k.feature = -1;
    k.threshold = 0;
    k.group = k.offset = k.num_bin = k.mfb = k.default_bin = 0;
    k.missing = k.default_left = k.is_cat = k.pad0 = 0;
    k.pos = a.rank * a.Fmax + j;
    k.pad2 = 0;
    s_key[t] = k;
  }
  if (t == 0 && j == 0 && c.num_leaves == 1) {
    // root output (every rank: the host reads it back with the tree)
    SplitParams p0 = a.sp;
    p0.path_smooth = 0.0;
    a.lout[0] = LeafOutputRaw(a.lsum[0].x, a.lsum[0].y, p0, a.gcount[0], 0.0);
  }
  if (f >= 0) {
    // Loads that do not depend on the histogram are issued first so their latency hides
    // under the fold: slots of the two children, the parent (larger child's slot) values
    // this thread subtracts, the leaf statistics the scanning waves read (held by lane 0
    // of waves 0 / 1 until used) and the feature masks.
    const int s_slot = a.slot[c.smaller];
    const int l_slot = c.larger >= 0 ? a.slot[c.larger] : -1;
    const DevFeature fi = a.feat[f];
    const int nbin = fi.num_bin;
    const int nst = nbin - 1;
    const int nv = 2 * nst;  // stored values of this feature
    const size_t slot_stride = 2 * static_cast<size_t>(a.TB);
    const size_t v0 = 2 * static_cast<size_t>(fi.hist_offset);
    double* gs = a.slots + s_slot * slot_stride + v0;
    double* gl = l_slot >= 0 ? a.slots + l_slot * slot_stride + v0 : nullptr;
    constexpr int kPre = 2;  // parent values per thread held in registers (nv <= kPre * blockDim)
    double parent[kPre];
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
      const int v = t + k * kScanThreads;
      parent[k] = (gl && v < nv) ? gl[v] : 0.0;
    }
    const int my_leaf = (w == 0) ? c.smaller : (w == 1 ? c.larger : -1);
    double2 pre_sum = make_double2(0.0, 0.0);
    int pre_n = 0, pre_depth = 0;
    double pre_out = 0.0;
    LeafBounds pre_bounds;
    if (lane == 0 && my_leaf >= 0) {
      pre_sum = a.lsum[my_leaf];
      pre_n = a.vote ? a.range[my_leaf].count : a.gcount[my_leaf];
      pre_out = a.lout[my_leaf];
      pre_bounds = a.bounds[my_leaf];
      pre_depth = a.depth[my_leaf];
    }
    int pre_used = 1, pre_spl = 1;
    if (t == 0) {
      pre_used = a.used_bytree[f];
      // the voting learner's local pass tries every feature (no splittable inheritance)
      pre_spl = (c.larger >= 0 && !a.vote) ? a.splittable[static_cast<size_t>(s_slot) * a.F + f] : 1;
    }
    double* hs_full = reinterpret_cast<double*>(smem);                 // 2 * nbin: smaller child, full
    double* hl_full = hs_full + 2 * a.max_bin;                          // 2 * nbin: larger child, full
    double* part = hl_full + 2 * a.max_bin;                             // [16][64]
    int* order = reinterpret_cast<int*>(part + 16 * 64);                // [2][cat_p2] categorical scratch
    double* ckey = reinterpret_cast<double*>(order + 2 * a.cat_p2);     // [2][cat_p2] ctr sort keys
    (void)part;
    const int n_small = a.range[c.smaller].count;
    // 1. smaller child's histogram into hs_full at stored positions (mfb filled in step 3)
    if (a.scan_src == 1) {
      // the owner row the data-parallel reduce-scatter delivered (2 * bbin values)
      const Acc* rows = reinterpret_cast<const Acc*>(a.rx) + 2 * static_cast<size_t>(fi.hist_offset - a.own_bin0);
      for (int v = t; v < nv; v += blockDim.x) {
        const double acc = static_cast<double>(rows[v]);
        const int k = v >> 1;
        const int b = k < fi.mfb ? k : k + 1;
        hs_full[2 * b + (v & 1)] = acc;
      }
    } else {
      const int nb = c.hist_nb > 0 ? c.hist_nb : HistActiveBlocks(n_small, hist_grid, a.hist_min_rows);
      const size_t V = 2 * static_cast<size_t>(a.TB);
      const size_t v0 = 2 * static_cast<size_t>(fi.hist_offset);
      const Acc* slab = reinterpret_cast<const Acc*>(a.hist_slab);
      // each wave owns 32 values, its two half-waves stride over the slab rows;
      // no barrier until all values are reduced
#if LGAP_SCAN_FOLD == 2
      // 16-lane quarter-waves each own 32 values as 16 pairs (one 2-element load per row) and
      // stride over the slab rows 4 apart: half the dependent loads per lane of the half-wave form
      const int quarter = lane >> 4, q = lane & 15;
      for (int vbase = w * 32; vbase < nv; vbase += (kScanThreads / 64) * 32) {
        const int v = vbase + 2 * q;  // nv is even, so v < nv implies v + 1 < nv
        double acc0 = 0.0, acc1 = 0.0;
        if (v < nv) {
          const Acc* col = slab + v0 + v;
#pragma unroll LGAP_SCAN_UNROLL
          for (int p = quarter; p < nb; p += 4) {
            const Acc* e = col + static_cast<size_t>(p) * V;
            acc0 += static_cast<double>(e[0]);
            acc1 += static_cast<double>(e[1]);
          }
        }
        acc0 += __shfl_xor(acc0, 16, kWave);
        acc1 += __shfl_xor(acc1, 16, kWave);
        acc0 += __shfl_xor(acc0, 32, kWave);
        acc1 += __shfl_xor(acc1, 32, kWave);
        if (lane < 16 && v < nv) {
          const int k = v >> 1;  // (v, v + 1) are the (grad, hess) of stored bin k
          const int b = k < fi.mfb ? k : k + 1;
          hs_full[2 * b] = acc0;
          hs_full[2 * b + 1] = acc1;
        }
      }
#else
      const int half = lane >> 5;
      // this block's run of slab rows (all of them unless the fold is split)
      const int p0 = C > 1 ? static_cast<int>((static_cast<long long>(ch) * nb) / C) : 0;
      const int p1 = C > 1 ? static_cast<int>((static_cast<long long>(ch + 1) * nb) / C) : nb;
      double* run = C > 1 ? a.fold_part + static_cast<size_t>(ch) * V + v0 : nullptr;
      for (int vbase = w * 32; vbase < nv; vbase += (kScanThreads / 64) * 32) {
        const int v = vbase + (lane & 31);
        double acc = 0.0;
        if (v < nv) {
          const Acc* col = slab + v0 + v;
#pragma unroll LGAP_SCAN_UNROLL
          for (int p = p0 + half; p < p1; p += 2) acc += static_cast<double>(col[static_cast<size_t>(p) * V]);
        }
        acc += __shfl_xor(acc, 32, kWave);
        if (lane < 32 && v < nv) {
          if (run) {
            run[v] = acc;
          } else {
            const int k = v >> 1;
            const int b = k < fi.mfb ? k : k + 1;
            hs_full[2 * b + (v & 1)] = acc;
          }
        }
      }
      if (C > 1) {
        // in-launch combine (one agent release per block, one acquire in the last arriver):
        // runs stored -> release -> ticket; the block drawing the last ticket of this launch
        // acquires and sums the C runs in chunk order (deterministic)
        __shared__ int s_last;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          const unsigned old = __hip_atomic_fetch_add(&a.fold_cnt[j], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_last = (old % static_cast<unsigned>(C)) == static_cast<unsigned>(C - 1) ? 1 : 0;
        }
        __syncthreads();
        if (!s_last) return;
        if (t == 0) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        const double* runs = a.fold_part + v0;
        for (int v = t; v < nv; v += blockDim.x) {
          double acc = 0.0;
          for (int r = 0; r < C; ++r) acc += runs[static_cast<size_t>(r) * V + v];
          const int k = v >> 1;
          const int b = k < fi.mfb ? k : k + 1;
          hs_full[2 * b + (v & 1)] = acc;
        }
      }
#endif
    }
    __syncthreads();
    Stamp(a, 3, 1);
    // 2. slots: smaller <- reduced; larger <- parent - smaller
    auto slot_update = [&](int v, double pv) {
      const int k = v >> 1;
      const int b = k < fi.mfb ? k : k + 1;
      const double sv = hs_full[2 * b + (v & 1)];
      gs[v] = sv;
      if (gl) {
        const double lv = pv - sv;
        gl[v] = lv;
        hl_full[2 * b + (v & 1)] = lv;
      }
    };
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
      const int v = t + k * kScanThreads;
      if (v < nv) slot_update(v, parent[k]);
    }
    for (int v = t + kPre * kScanThreads; v < nv; v += kScanThreads) slot_update(v, gl ? gl[v] : 0.0);
    if (t == 0) {
      const bool skip_both = !pre_used || !pre_spl;
      s_skip_both = skip_both ? 1 : 0;
      // extra-trees draws in the host learner's order: smaller leaf first, then larger
      s_rand[0] = s_rand[1] = 0;
      if (a.sp.extra_trees && !skip_both && fi.bin_type == 0 && fi.num_bin - 2 > 0) {
        s_rand[0] = RandNextInt(&a.rng[f], 0, fi.num_bin - 2);
        if (c.larger >= 0) s_rand[1] = RandNextInt(&a.rng[f], 0, fi.num_bin - 2);
      }
    }
    __syncthreads();
    Stamp(a, 3, 2);
    // 3. most-frequent bin = leaf total - stored bins
    if (w < 2) {
      const int leaf = w == 0 ? c.smaller : c.larger;
      if (leaf >= 0) {
        double* H = w == 0 ? hs_full : hl_full;
        double sgs = 0.0, shs = 0.0;
        for (int b = lane; b < nbin; b += 64) {
          if (b == fi.mfb) continue;
          sgs += H[2 * b];
          shs += H[2 * b + 1];
        }
        sgs = WaveSum(sgs);
        shs = WaveSum(shs);
        double2 sums = pre_sum;  // lane 0's prefetched leaf sums (only lane 0 uses them)
        if (a.vote) {
          // voting local pass: the smaller child's local sums are the k_hist row sums; the
          // larger child's are the split leaf's local sums (Ctl) minus them
          const int nbp = HistActiveBlocks(n_small, hist_grid, a.hist_min_rows);
          double pg = 0.0, ph = 0.0;
          for (int p = lane; p < nbp; p += 64) {
            const double2 x = a.hsum_part[p];
            pg += x.x;
            ph += x.y;
          }
          pg = WaveSum(pg);
          ph = WaveSum(ph);
          sums = w == 0 ? make_double2(pg, ph) : make_double2(c.plg - pg, c.plh - ph);
          if (j == 0 && lane == 0) a.lsum_loc[leaf] = sums;
        }
        if (lane == 0) {
          H[2 * fi.mfb] = sums.x - sgs;
          H[2 * fi.mfb + 1] = sums.y - shs;
          s_sum[w][0] = sums.x;
          s_sum[w][1] = sums.y;
        }
      }
    }
    __syncthreads();
    Stamp(a, 3, 3);
    const int sel = w;
    const int leaf = sel == 0 ? c.smaller : c.larger;
    if (w < 2 && leaf >= 0) {
      SplitInfo* out = &s_out[sel];  // built in LDS, published by the whole block below
      if (!s_skip_both) {
        const double* H = sel ? hl_full : hs_full;
        const int lslot = sel ? l_slot : s_slot;
        const double sg = s_sum[sel][0], sh = s_sum[sel][1];
        const int n = __shfl(pre_n, 0, kWave);
        double po;
        if (c.num_leaves == 1) {
          SplitParams p0 = a.sp;
          p0.path_smooth = 0.0;
          po = LeafOutputRaw(sg, sh, p0, n, 0.0);
        } else {
          po = __shfl(pre_out, 0, kWave);
        }
        LeafBounds bounds;
        bounds.min = __shfl(pre_bounds.min, 0, kWave);
        bounds.max = __shfl(pre_bounds.max, 0, kWave);
        const int depth = __shfl(pre_depth, 0, kWave);
        bool sp;
        if (fi.bin_type == 0) {
          sp = ScanNumericalWave(a.sp, fi, H, sg, sh, n, po, bounds, s_rand[sel], out);
        } else {
          // categorical: the wave-parallel one-hot / ctr-sorted scan
          FeatureScanMeta m;
          m.num_bin = fi.num_bin;
          m.default_bin = static_cast<uint32_t>(fi.default_bin);
          m.missing_type = fi.missing;
          m.bin_type = fi.bin_type;
          m.monotone = fi.monotone;
          m.penalty = fi.penalty;
          int rt = 0;
          if (a.sp.extra_trees && lane == 0) {
            // (categorical draws happen here; numerical ones were drawn above)
            if (fi.num_bin <= a.sp.max_cat_to_onehot) {
              if (fi.num_bin - 1 > 0) rt = RandNextInt(&a.rng[f], 1, fi.num_bin);
            } else {
              const double cf = n / (sh + 2 * kEpsilon);
              int used = 0;
              for (int b = 1; b < fi.num_bin; ++b) used += RoundCount(H[2 * b + 1] * cf) >= a.sp.cat_smooth;
              const int max_num_cat = min(a.sp.max_cat_threshold, (used + 1) / 2);
              const int max_thr = max(min(max_num_cat, used) - 1, 0);
              if (max_thr > 0) rt = RandNextInt(&a.rng[f], 0, max_thr);
            }
          }
          m.rand_threshold = __shfl(rt, 0, kWave);
          if (lane == 0) out->Reset();
          sp = ScanCategoricalWave(a.sp, m, H, sg, sh, n, po, bounds, a.cat_p2, order + sel * a.cat_p2,
                                   ckey + sel * a.cat_p2, out);
        }
        if (lane == 0) {
          if (!a.vote) a.splittable[static_cast<size_t>(lslot) * a.F + f] = sp ? 1 : 0;
          if (!sp) {
            out->Reset();
          } else {
            out->feature = f;
            // (the voting learner's local pass ranks raw gains: penalties and node masks
            // apply in its global pass, k_vote_scan)
            if (!a.vote) {
              // cost-effective gradient boosting, split penalty (host CegbPenalty::DeltaGain:
              // subtracted before the monotone penalty multiplies the gain)
              if (a.cegb_split > 0.0) out->gain -= a.cegb_split * n;
              if (out->monotone_type != 0) out->gain *= MonotonePenaltyAt(a.monotone_penalty, depth);
              if (a.bynode && !a.bynode[static_cast<size_t>(c.scan_round == 0 ? 0 : 2 * c.scan_round - 1 + sel) * a.F + f]) out->Reset();
              if (a.ic_feat && (a.ic_leaf[leaf] & a.ic_feat[f]) == 0ull) out->Reset();
            }
          }
        }
      }
      if (lane == 0) {
        // the compact candidate the partition's select reads
        SplitKey& k = s_key[sel];
        k.feature = out->feature;
        k.gain = SafeGain(*out);
        k.threshold = out->threshold;
        k.group = fi.group;
        k.offset = fi.offset;
        k.num_bin = fi.num_bin;
        k.mfb = fi.mfb;
        k.default_bin = fi.default_bin;
        k.missing = fi.missing;
        k.default_left = out->default_left;
        k.is_cat = fi.bin_type != 0 ? 1 : 0;
      }
    }
  }
  __syncthreads();
  // 4. publish the two candidates (dword-parallel copies of the LDS records)
  {
    constexpr int kKeyWords = static_cast<int>(sizeof(SplitKey) / 4);
    constexpr int kInfoWords = static_cast<int>(sizeof(SplitInfo) / 4);
    constexpr int kWords = 2 * (kKeyWords + kInfoWords);
    {
      char* tbl = a.cand;
      for (int i = t; i < kWords; i += blockDim.x) {
        const int sel = i / (kKeyWords + kInfoWords);
        const int o = i - sel * (kKeyWords + kInfoWords);
        char* blk = tbl + static_cast<size_t>(a.rank) * a.cand_stride;
        if (o < kKeyWords) {
          reinterpret_cast<uint32_t*>(reinterpret_cast<SplitKey*>(blk) + sel * a.Fmax + j)[o] =
              reinterpret_cast<const uint32_t*>(&s_key[sel])[o];
        } else {
          reinterpret_cast<uint32_t*>(reinterpret_cast<SplitInfo*>(blk + a.cand_key_bytes) + sel * a.Fmax + j)[o - kKeyWords] =
              reinterpret_cast<const uint32_t*>(&s_out[sel])[o - kKeyWords];
        }
      }
    }
  }
  Stamp(a, 3, 4);
  if (t == 0 && a.stamps) {
    atomicMax(&a.stamps[((static_cast<size_t>(3) * 256 + (a.ctl->num_splits & 255)) * 2) * 8 + 7], wall_clock64());
  }
}

// ---------------------------------------------------------------------------
// Voting parallel (PV-Tree; reference voting_parallel_tree_learner.cpp:243-399), on the
// device. Rows are sharded like data parallel, but the per-split exchange carries only
// what the vote needs:
//   k_hist        local histogram of the smaller child (+ its local (sum g, sum h))
//   k_reduce_scan LOCAL pass over every feature: local sums / counts, min_data and
//                 min_sum_hessian divided by the ranks -> local candidate table
//   k_vote_local  this rank's top-k per child -> VoteRec rows, all-gathered (xGMI push
//                 + in-kernel exchange, or ncclAllGather)
//   k_vote_pack   every block elects the same <= top_k features per child from the
//                 gathered rows (GlobalVoting: gain weighted by count / mean leaf count,
//                 best record per feature, top_k), and packs this rank's local histogram
//                 of one elected feature; the packed rows are summed over the ranks
//                 (xGMI push + in-kernel exchange, or ncclAllReduce)
//   k_vote_scan   GLOBAL pass over the elected features only (global sums and counts,
//                 split penalties, node masks) -> the candidate table the partition's
//                 select reads. Every rank computes the same table: no further exchange.
// The local histograms stay in the slots (parent - smaller subtraction stays local).


// instantiations launched by the DeviceTreeLearner
template __global__ void k_reduce_scan<double, false>(Args, int);
template __global__ void k_reduce_scan<double, true>(Args, int);
template __global__ void k_reduce_scan<float, false>(Args, int);
template __global__ void k_reduce_scan<float, true>(Args, int);

}  // namespace seq
}  // namespace device
}  // namespace lgap
