// Per-row gradient / hessian formulas of every pointwise objective, shared by
// the host objectives and the HIP gradient kernel so both paths compute the
// same numbers (formulas: reference regression_objective.hpp:132-745,
// binary_objective.hpp:105-136, xentropy_objective.hpp:105-250).
#pragma once

#include <cmath>

#include "lgap/meta.h"

namespace lgap {

enum PointwiseKind : int {
  kPwL2 = 0,
  kPwL1 = 1,
  kPwHuber = 2,
  kPwFair = 3,
  kPwPoisson = 4,
  kPwQuantile = 5,
  kPwMape = 6,
  kPwGamma = 7,
  kPwTweedie = 8,
  kPwBinary = 9,
  kPwXent = 10,
  kPwXentLambda = 11,
};

struct PointwiseParams {
  int kind = kPwL2;
  double alpha = 0.9;         // huber / quantile
  double fair_c = 1.0;
  double exp_max_delta = 1.0; // poisson: exp(poisson_max_delta_step)
  double rho = 1.5;           // tweedie
  double sigmoid = 1.0;       // binary
  double label_weight_neg = 1.0, label_weight_pos = 1.0;  // binary unbalance / scale_pos_weight
};

LGAP_HD inline double PwSign(double x) { return (x > 0.0) - (x < 0.0); }

// `w` is the row weight (1 when the dataset is unweighted; `weighted` selects
// the reference's weighted code path where it differs numerically).
// `aux` is the MAPE label weight 1/max(1,|y|) (already multiplied by w).
LGAP_HD inline void PointwiseGradient(const PointwiseParams& p, double s, double y, double w, bool weighted, double aux,
                                      score_t* g, score_t* h) {
  switch (p.kind) {
    case kPwL2:
      if (weighted) {
        *g = static_cast<score_t>(static_cast<score_t>(s - y) * w);
        *h = static_cast<score_t>(w);
      } else {
        *g = static_cast<score_t>(s - y);
        *h = 1.0f;
      }
      break;
    case kPwL1: {
      const double d = s - y;
      *g = static_cast<score_t>(PwSign(d) * w);
      *h = static_cast<score_t>(w);
      break;
    }
    case kPwHuber: {
      const double d = s - y;
      const double gg = fabs(d) <= p.alpha ? d : PwSign(d) * p.alpha;
      *g = static_cast<score_t>(gg * w);
      *h = static_cast<score_t>(w);
      break;
    }
    case kPwFair: {
      const double x = s - y;
      const double den = fabs(x) + p.fair_c;
      *g = static_cast<score_t>(p.fair_c * x / den * w);
      *h = static_cast<score_t>(p.fair_c * p.fair_c / (den * den) * w);
      break;
    }
    case kPwPoisson: {
      const double e = exp(s);
      *g = static_cast<score_t>((e - y) * w);
      *h = static_cast<score_t>(e * p.exp_max_delta * w);
      break;
    }
    case kPwQuantile: {
      const double d = s - y;
      const double gg = d >= 0.0 ? (1.0 - p.alpha) : -p.alpha;
      *g = static_cast<score_t>(gg * w);
      *h = static_cast<score_t>(w);
      break;
    }
    case kPwMape: {
      const double d = s - y;
      *g = static_cast<score_t>(PwSign(d) * aux);
      *h = static_cast<score_t>(w);
      break;
    }
    case kPwGamma: {
      const double e = exp(-s);
      *g = static_cast<score_t>((1.0 - y * e) * w);
      *h = static_cast<score_t>(y * e * w);
      break;
    }
    case kPwTweedie: {
      const double e1 = exp((1.0 - p.rho) * s);
      const double e2 = exp((2.0 - p.rho) * s);
      *g = static_cast<score_t>((-y * e1 + e2) * w);
      *h = static_cast<score_t>((-y * (1.0 - p.rho) * e1 + (2.0 - p.rho) * e2) * w);
      break;
    }
    case kPwBinary: {
      const bool pos = y > 0;
      const int lab = pos ? 1 : -1;
      const double lw = pos ? p.label_weight_pos : p.label_weight_neg;
      const double r = -lab * p.sigmoid / (1.0f + exp(lab * p.sigmoid * s));
      const double ar = fabs(r);
      *g = static_cast<score_t>(r * lw * w);
      *h = static_cast<score_t>(ar * (p.sigmoid - ar) * lw * w);
      break;
    }
    case kPwXent: {
      if (s > -37.0) {
        const double e = exp(-s);
        *g = static_cast<score_t>(((1.0f - y) - y * e) / (1.0f + e) * w);
        *h = static_cast<score_t>(e / ((1 + e) * (1 + e)) * w);
      } else {
        const double e = exp(s);
        *g = static_cast<score_t>((e - y) * w);
        *h = static_cast<score_t>(e * w);
      }
      break;
    }
    case kPwXentLambda: {
      if (!weighted) {
        const double z = 1.0f / (1.0f + exp(-s));
        *g = static_cast<score_t>(z - y);
        *h = static_cast<score_t>(z * (1.0f - z));
      } else {
        const double epf = exp(s);
        const double hhat = log1p(epf);
        const double z = 1.0f - exp(-w * hhat);
        const double enf = 1.0f / epf;
        *g = static_cast<score_t>((1.0f - y / z) * w / (1.0f + enf));
        const double c = 1.0f / (1.0f - z);
        double d = 1.0f + epf;
        const double a = w * epf / (d * d);
        d = c - 1.0f;
        const double b = (c / (d * d)) * (1.0f + w * epf - c);
        *h = static_cast<score_t>(a * (1.0f + y * b));
      }
      break;
    }
    default:
      *g = 0.0f;
      *h = 0.0f;
  }
}

}  // namespace lgap
