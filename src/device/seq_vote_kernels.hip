// Sequential chain, voting parallel (PV-Tree): local scan, top-k election, elected-histogram
// scan; leaf true sums for quantized training (declarations: seq_kernels.h).
#include "device/seq_kernels.h"

namespace lgap {
namespace device {
namespace seq {


// best record first: higher gain, then smaller feature (SplitInfo::BetterThan)
__device__ __forceinline__ bool VoteBetter(double ga, int fa, double gb, int fb) {
  return ga != gb ? ga > gb : fa < fb;
}

__global__ __launch_bounds__(kVoteThreads) void k_vote_local(Args a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const Ctl c = *a.ctl;
  if (c.done || c.skip) return;
  const int F = a.F, K = a.topk, t = threadIdx.x;
  double* s_gain = reinterpret_cast<double*>(smem);
  int* s_cnt = reinterpret_cast<int*>(s_gain + F);
  __shared__ int s_n[kVoteThreads / 64];
  const SplitKey* keys = reinterpret_cast<const SplitKey*>(a.lcand);
  const SplitInfo* infos = reinterpret_cast<const SplitInfo*>(a.lcand + a.lcand_key_bytes);
  for (int sel = 0; sel < 2; ++sel) {
    const int leaf = sel ? c.larger : c.smaller;
    int nv = 0;
    for (int f = t; f < F; f += blockDim.x) {
      const SplitKey k = keys[sel * F + f];
      const bool valid = leaf >= 0 && k.feature >= 0;
      s_gain[f] = valid ? k.gain : kMinScore;
      s_cnt[f] = valid ? infos[sel * F + f].left_count + infos[sel * F + f].right_count : -1;
      nv += valid ? 1 : 0;
    }
    const int nvalid = BlockSumInt(nv, s_n);  // (barrier inside: the LDS arrays are complete)
    for (int f = t; f < F; f += blockDim.x) {
      if (s_cnt[f] < 0) continue;
      const double g = s_gain[f];
      int rank = 0;
      for (int j = 0; j < F && rank < K; ++j) rank += (s_cnt[j] >= 0 && VoteBetter(s_gain[j], j, g, f)) ? 1 : 0;
      if (rank < K) {
        VoteRec r;
        r.gain = g;
        r.feature = f;
        r.count = s_cnt[f];
        a.vrec[static_cast<size_t>(a.rank) * 2 * K + sel * K + rank] = r;
      }
    }
    for (int i = nvalid + t; i < K; i += blockDim.x) {
      VoteRec r;
      r.gain = kMinScore;
      r.feature = -1;
      r.count = 0;
      a.vrec[static_cast<size_t>(a.rank) * 2 * K + sel * K + i] = r;
    }
    __syncthreads();
  }
}

// GlobalVoting of child `sel` over the gathered rows (same result in every block and on
// every rank): s_list[0..n) = the elected features in ascending order; returns n.
__device__ int ElectChild(const Args& a, const Ctl& c, int sel, const VoteRec* recs, double* s_w, int* s_f,
                          int* s_flag, int* s_list, int* s_tmp) {
  const int K = a.topk, R = a.P * K, t = threadIdx.x;
  const int leaf = sel ? c.larger : c.smaller;
  // mean leaf count per rank in float, as the reference's score_t mean_num_data
  const float mean = leaf >= 0 ? static_cast<float>(a.gcount[leaf]) / static_cast<float>(a.P) : 1.f;
  for (int i = t; i < R; i += blockDim.x) {
    const int r = i / K, k = i - r * K;
    const VoteRec v = recs[static_cast<size_t>(r) * 2 * K + sel * K + k];
    const double w = v.gain * v.count / static_cast<double>(mean);
    const bool valid = leaf >= 0 && v.feature >= 0 && w > kMinScore;
    s_w[i] = w;
    s_f[i] = valid ? v.feature : -1;
  }
  __syncthreads();
  // the best record of each feature (first in gather order on equal weighted gain)
  for (int i = t; i < R; i += blockDim.x) {
    int best = s_f[i] >= 0 ? 1 : 0;
    for (int j = 0; j < R && best; ++j) {
      if (j != i && s_f[j] == s_f[i] && (s_w[j] > s_w[i] || (s_w[j] == s_w[i] && j < i))) best = 0;
    }
    s_flag[i] = best;
  }
  __syncthreads();
  // elected: feature-best records ranked < K by (weighted gain desc, feature asc)
  int ne = 0;
  for (int i = t; i < R; i += blockDim.x) {
    int el = 0;
    if (s_flag[i]) {
      int rank = 0;
      for (int j = 0; j < R && rank < K; ++j) rank += (s_flag[j] && VoteBetter(s_w[j], s_f[j], s_w[i], s_f[i])) ? 1 : 0;
      el = rank < K ? 1 : 0;
    }
    ne += el;
    s_tmp[i] = el;
  }
  __syncthreads();
  for (int i = t; i < R; i += blockDim.x) s_flag[i] = s_tmp[i];
  const int n = BlockSumInt(ne, s_tmp + R);
  for (int i = t; i < R; i += blockDim.x) {
    if (!s_flag[i]) continue;
    int pos = 0;
    for (int j = 0; j < R; ++j) pos += (s_flag[j] && s_f[j] < s_f[i]) ? 1 : 0;
    s_list[pos] = s_f[i];
  }
  __syncthreads();
  return n;
}

__device__ __forceinline__ int VoteValues(const Args& a, int f) { return 2 * (a.feat[f].num_bin - 1); }

// One block per (child, elected rank): elect (redundantly per block), then pack this
// rank's local histogram of the block's feature into the packed row at its offset.
template <typename Acc>
__global__ __launch_bounds__(kVoteThreads) void k_vote_pack(Args a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const Ctl c = *a.ctl;
  if (c.done || c.skip) return;
  const int K = a.topk, R = a.P * K, t = threadIdx.x;
  double* s_w = reinterpret_cast<double*>(smem);
  int* s_f = reinterpret_cast<int*>(s_w + R);
  int* s_flag = s_f + R;
  int* s_tmp = s_flag + R;                     // R + kVoteThreads / 64
  int* s_list = s_tmp + R + kVoteThreads / 64;  // [2][K]
  __shared__ int s_n[2];
  const VoteRec* recs = a.vrec;
  for (int sel = 0; sel < 2; ++sel) {
    const int n = ElectChild(a, c, sel, recs, s_w, s_f, s_flag, s_list + sel * K, s_tmp);
    if (t == 0) s_n[sel] = n;
    __syncthreads();
  }
  const int sel = blockIdx.x / K, k = blockIdx.x - sel * K;
  int base0 = 0;
  for (int i = 0; i < s_n[0]; ++i) base0 += VoteValues(a, s_list[i]);
  if (blockIdx.x == 0 && t < 2) {
    int* e = a.elect + t * (K + 2);
    e[0] = s_n[t];
    e[1] = t == 0 ? 0 : base0;
  }
  if (blockIdx.x == 0) {
    for (int i = t; i < 2 * K; i += blockDim.x) {
      const int sl = i / K, kk = i - sl * K;
      a.elect[sl * (K + 2) + 2 + kk] = kk < s_n[sl] ? s_list[sl * K + kk] : -1;
    }
  }
  const int leaf = sel ? c.larger : c.smaller;
  if (k < s_n[sel] && leaf >= 0) {
    const int f = s_list[sel * K + k];
    int off = sel ? base0 : 0;
    for (int i = 0; i < k; ++i) off += VoteValues(a, s_list[sel * K + i]);
    const int nv = VoteValues(a, f);
    const double* src = a.slots + static_cast<size_t>(a.slot[leaf]) * 2 * a.TB + 2 * static_cast<size_t>(a.feat[f].hist_offset);
    for (int v = t; v < nv; v += blockDim.x) {
      reinterpret_cast<Acc*>(a.vhist)[off + v] = static_cast<Acc>(src[v]);
    }
  }
}

// Global pass: block k, wave `sel` scans elected feature k of child sel from the summed
// packed rows with the GLOBAL leaf statistics; writes the candidate table (one row of
// 2 x top_k positions) that the partition's select reads.
template <typename Acc, bool kGlobal>
__global__ __launch_bounds__(128) void k_vote_scan(Args a) {
  extern __shared__ __align__(16) unsigned char smem_dyn[];
  // (kGlobal launches never split the fold: blockIdx.x is the feature slot)
  unsigned char* smem = kGlobal ? reinterpret_cast<unsigned char*>(a.scan_scratch) + blockIdx.x * a.scan_scratch_stride
                                : smem_dyn;
  const Ctl c = *a.ctl;
  if (c.done || c.skip) return;
  const int K = a.topk, k = blockIdx.x, t = threadIdx.x, lane = t & 63, sel = t >> 6;
  __shared__ __align__(8) unsigned char s_out_raw[2 * sizeof(SplitInfo)];
  SplitInfo* out = reinterpret_cast<SplitInfo*>(s_out_raw) + sel;
  double* H = reinterpret_cast<double*>(smem) + sel * 2 * a.max_bin;
  int* order = reinterpret_cast<int*>(reinterpret_cast<double*>(smem) + 4 * a.max_bin) + sel * a.cat_p2;
  double* ckey = reinterpret_cast<double*>(reinterpret_cast<int*>(reinterpret_cast<double*>(smem) + 4 * a.max_bin) +
                                           2 * a.cat_p2) + sel * a.cat_p2;
  const int* e = a.elect + sel * (K + 2);
  const int leaf = sel ? c.larger : c.smaller;
  SplitKey key;
  key.gain = kMinScore;
  key.feature = -1;
  key.threshold = 0;
  key.group = key.offset = key.num_bin = key.mfb = key.default_bin = 0;
  key.missing = key.default_left = key.is_cat = key.pad0 = 0;
  key.pos = k;  // table row 0, column k of child sel (CandInfoPos(a, sel, k))
  key.pad2 = 0;
  if (lane == 0) out->Reset();
  if (leaf >= 0 && k < e[0]) {
    const int f = e[2 + k];
    const DevFeature fi = a.feat[f];
    int off = e[1];
    for (int i = 0; i < k; ++i) off += VoteValues(a, e[2 + i]);
    const int nv = 2 * (fi.num_bin - 1);
    const Acc* rows = reinterpret_cast<const Acc*>(a.vhist);
    double sgs = 0.0, shs = 0.0;
    for (int v = lane; v < nv; v += 64) {
      const double acc = static_cast<double>(rows[off + v]);
      const int kb = v >> 1;
      const int b = kb < fi.mfb ? kb : kb + 1;
      H[2 * b + (v & 1)] = acc;
      if (v & 1) shs += acc;
      else sgs += acc;
    }
    sgs = WaveSum(sgs);
    shs = WaveSum(shs);
    const double2 sums = a.lsum[leaf];
    const int n = a.gcount[leaf];
    if (lane == 0) {
      H[2 * fi.mfb] = sums.x - sgs;
      H[2 * fi.mfb + 1] = sums.y - shs;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    double po;
    if (c.num_leaves == 1) {
      SplitParams p0 = a.sp;
      p0.path_smooth = 0.0;
      po = LeafOutputRaw(sums.x, sums.y, p0, n, 0.0);
    } else {
      po = a.lout[leaf];
    }
    const LeafBounds bounds = a.bounds[leaf];
    bool sp;
    if (fi.bin_type == 0) {
      sp = ScanNumericalWave(a.sp, fi, H, sums.x, sums.y, n, po, bounds, 0, out);
    } else {
      FeatureScanMeta m;
      m.num_bin = fi.num_bin;
      m.default_bin = static_cast<uint32_t>(fi.default_bin);
      m.missing_type = fi.missing;
      m.bin_type = fi.bin_type;
      m.monotone = fi.monotone;
      m.penalty = fi.penalty;
      m.rand_threshold = 0;
      if (lane == 0) out->Reset();
      sp = ScanCategoricalWave(a.sp, m, H, sums.x, sums.y, n, po, bounds, a.cat_p2, order, ckey, out);
    }
    if (lane == 0) {
      if (!sp) {
        out->Reset();
      } else {
        out->feature = f;
        if (out->monotone_type != 0) out->gain *= MonotonePenaltyAt(a.monotone_penalty, a.depth[leaf]);
        if (a.bynode && !a.bynode[static_cast<size_t>(c.scan_round == 0 ? 0 : 2 * c.scan_round - 1 + sel) * a.F + f]) out->Reset();
        if (a.ic_feat && (a.ic_leaf[leaf] & a.ic_feat[f]) == 0ull) out->Reset();
      }
      key.feature = out->feature;
      key.gain = SafeGain(*out);
      key.threshold = out->threshold;
      key.group = fi.group;
      key.offset = fi.offset;
      key.num_bin = fi.num_bin;
      key.mfb = fi.mfb;
      key.default_bin = fi.default_bin;
      key.missing = fi.missing;
      key.default_left = out->default_left;
      key.is_cat = fi.bin_type != 0 ? 1 : 0;
    }
  }
  __syncthreads();
  if (lane == 0) *CandKey(a, 0, sel, k) = key;
  constexpr int kInfoWords = static_cast<int>(sizeof(SplitInfo) / 4);
  for (int i = lane; i < kInfoWords; i += 64) {
    reinterpret_cast<uint32_t*>(CandInfo(a, 0, sel, k))[i] = reinterpret_cast<const uint32_t*>(out)[i];
  }
}

// quant_train_renew_leaf: per-leaf sums of the unquantized (g, h); one block per leaf
__global__ __launch_bounds__(kNodeThreads) void k_leaf_true_sums(Args a, const float2* gh_true, int num_leaves,
                                                                  double2* out) {
  __shared__ double sh[2][kNodeThreads / 64];
  const int leaf = blockIdx.x;
  if (leaf >= num_leaves) return;
  const LeafRange r = a.range[leaf];
  double g = 0.0, h = 0.0;
  for (int i = threadIdx.x; i < r.count; i += blockDim.x) {
    const float2 v = gh_true[RowAt(a, r.buf, r.start + i)];
    g += v.x;
    h += v.y;
  }
  g = WaveSum(g);
  h = WaveSum(h);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[0][w] = g;
    sh[1][w] = h;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tg = 0.0, th = 0.0;
    for (int k = 0; k < kNodeThreads / 64; ++k) tg += sh[0][k], th += sh[1][k];
    out[leaf] = make_double2(tg, th);
  }
}

// Copy a SplitInfo with one dword per thread (no serial per-thread struct copy).

// instantiations launched by the DeviceTreeLearner
template __global__ void k_vote_pack<double>(Args);
template __global__ void k_vote_pack<float>(Args);
template __global__ void k_vote_scan<double, false>(Args);
template __global__ void k_vote_scan<double, true>(Args);
template __global__ void k_vote_scan<float, false>(Args);
template __global__ void k_vote_scan<float, true>(Args);

}  // namespace seq
}  // namespace device
}  // namespace lgap
