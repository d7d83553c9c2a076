// Per-row losses of the pointwise metrics and the objectives' output transforms,
// shared by the host metrics (src/metric/metrics.cpp) and the HIP metric kernel
// (src/device/grad_kernels.hip) so a training metric evaluated on the device
// equals the host's. Reference: regression_metric.hpp:20-320,
// binary_metric.hpp:20-190, xentropy_metric.hpp:20-330 (and the CUDA
// EvalKernel, metric/cuda/cuda_pointwise_metric.cu:20).
#pragma once

#include <cmath>

#include "lgap/meta.h"

namespace lgap {

enum PwMetricKind : int {
  kPmL2 = 0, kPmRmse, kPmL1, kPmQuantile, kPmHuber, kPmFair, kPmPoisson, kPmMape, kPmGamma, kPmGammaDev, kPmTweedie,
  kPmBinLogloss, kPmBinError, kPmXent, kPmXentLambda, kPmKldiv
};

// objective output transforms (ObjectiveFunction::ConvertOutput of the pointwise objectives)
enum PwOutput : int { kOutIdentity = 0, kOutSigmoid = 1, kOutExp = 2, kOutSignedSquare = 3, kOutLog1pExp = 4 };

struct PwMetricParams {
  int kind = kPmL2;
  double alpha = 0.9, fair_c = 1.0, tweedie_rho = 1.5;
  int output = kOutIdentity;
  double sigmoid = 1.0;  // kOutSigmoid: 1 / (1 + exp(-sigmoid * s))
};

LGAP_HD inline double PmConvert(const PwMetricParams& p, double s) {
  switch (p.output) {
    case kOutSigmoid: return 1.0f / (1.0f + exp(-p.sigmoid * s));
    case kOutExp: return exp(s);
    case kOutSignedSquare: return ((s > 0.0) - (s < 0.0)) * s * s;
    case kOutLog1pExp: return log1p(exp(s));
    default: return s;
  }
}

LGAP_HD inline double PmSafeLog(double x) { return x > 0 ? log(x) : -INFINITY; }

LGAP_HD inline double PmXent(double y, double p) {
  const double eps = 1.0e-12;
  const double a = y * (p > eps ? log(p) : log(eps));
  const double b = (1.0f - y) * (1.0f - p > eps ? log(1.0f - p) : log(eps));
  return -(a + b);
}

// loss of one row at converted score s (w only enters xentlambda's loss)
LGAP_HD inline double PmLoss(const PwMetricParams& p, double y, double s, double w) {
  switch (p.kind) {
    case kPmL2:
    case kPmRmse:
      return (s - y) * (s - y);
    case kPmL1:
      return fabs(s - y);
    case kPmQuantile: {
      const double d = y - s;
      return d < 0 ? (p.alpha - 1.0f) * d : p.alpha * d;
    }
    case kPmHuber: {
      const double d = s - y;
      return fabs(d) <= p.alpha ? 0.5f * d * d : p.alpha * (fabs(d) - 0.5f * p.alpha);
    }
    case kPmFair: {
      const double x = fabs(s - y), c = p.fair_c;
      return c * x - c * c * log1p(x / c);
    }
    case kPmPoisson:
      if (s < 1e-10f) s = 1e-10f;
      return s - y * log(s);
    case kPmMape:
      return fabs(y - s) / fmax(1.0, fabs(y));
    case kPmGamma: {
      const double theta = -1.0 / s;
      const double b = -PmSafeLog(-theta);
      const double c = PmSafeLog(y) - PmSafeLog(y);
      return -((y * theta - b) + c);
    }
    case kPmGammaDev: {
      const double t = y / (s + 1.0e-9);
      return t - PmSafeLog(t) - 1;
    }
    case kPmTweedie: {
      const double rho = p.tweedie_rho;
      if (s < 1e-10f) s = 1e-10f;
      const double a = y * exp((1 - rho) * log(s)) / (1 - rho);
      const double b = exp((2 - rho) * log(s)) / (2 - rho);
      return -a + b;
    }
    case kPmBinLogloss:
      if (y <= 0) {
        if (1.0f - s > kEpsilon) return -log(1.0f - s);
      } else if (s > kEpsilon) {
        return -log(s);
      }
      return -log(kEpsilon);
    case kPmBinError:
      return s <= 0.5f ? (y > 0) : (y <= 0);
    case kPmXent:
    case kPmKldiv:
      return PmXent(y, s);
    case kPmXentLambda:
      return PmXent(y, 1.0f - exp(-w * s));
  }
  return 0.0;
}

// weighted contribution of one row to the metric's sum (PointwiseMetric::Eval)
LGAP_HD inline double PmRowTerm(const PwMetricParams& p, double y, double raw, bool weighted, double w) {
  const double s = PmConvert(p, raw);
  if (p.kind == kPmXentLambda) return PmLoss(p, y, s, weighted ? w : 1.0);
  return weighted ? PmLoss(p, y, s, 1.0) * w : PmLoss(p, y, s, 1.0);
}

// Multiclass metrics (reference multiclass_metric.hpp:20-180): multi_logloss / multi_error@k
// of one row from its num_class raw scores (class-major, `stride` apart), through the
// objective's output transform: 0 raw (custom objective), 1 softmax (the host's
// common::Softmax order: max, exp-sum, divide), 2 one-vs-all sigmoids.
struct MultiMetricParams {
  int error = 0;      // 1: multi_error (top_k), 0: multi_logloss
  int top_k = 1;
  int output = 0;     // 0 raw, 1 softmax, 2 sigmoid per class
  double sigmoid = 1.0;
  int num_class = 0;
};

LGAP_HD inline double MultiProb(const MultiMetricParams& p, const double* s, size_t stride, int k, double wmax,
                                double sum) {
  const double x = s[static_cast<size_t>(k) * stride];
  if (p.output == 1) return exp(x - wmax) / sum;
  if (p.output == 2) return 1.0f / (1.0f + exp(-p.sigmoid * x));
  return x;
}

LGAP_HD inline double MultiRowLoss(const MultiMetricParams& p, const double* s, size_t stride, int y) {
  double wmax = 0.0, sum = 1.0;
  if (p.output == 1) {
    wmax = s[0];
    for (int k = 1; k < p.num_class; ++k) wmax = fmax(wmax, s[static_cast<size_t>(k) * stride]);
    sum = 0.0;
    for (int k = 0; k < p.num_class; ++k) sum += exp(s[static_cast<size_t>(k) * stride] - wmax);
  }
  const double py = MultiProb(p, s, stride, y, wmax, sum);
  if (p.error) {
    int larger = 0;
    for (int k = 0; k < p.num_class; ++k) {
      if (MultiProb(p, s, stride, k, wmax, sum) >= py && ++larger > p.top_k) return 1.0;
    }
    return 0.0;
  }
  return py > kEpsilon ? -log(py) : -log(kEpsilon);
}

}  // namespace lgap
