// Batched per-row constraint functions of the DRPO environments, evaluated on the
// device (replaces the three host numpy round trips per rollout step,
// src/smbpo.py:63-65). Numerics follow the reference: where numpy promotes to
// float64 (float64 constants / BoundedConstraint matrices) we compute in double,
// where it stays float32 (tracking geometry) we compute in float.
#pragma once
#include "common.hpp"

namespace drpo {

enum EnvId : int { ENV_POINT_ROBOT = 0, ENV_QUADROTOR = 1, ENV_CARTPOLE = 2, ENV_TRACKING = 3 };

struct EnvParams {
  int id;
  int surr_start;     // tracking: first surrounding-vehicle dim (47 for ref_num 1 / pre_horizon 10)
  int n_surr;         // tracking: number of surrounding vehicles
  double thr0, thr1;  // quadrotor: x/z_threshold (safe_control_gym, unpinned); cartpole: x/th_threshold
};

__host__ __device__ inline int env_con_dim(int id, int n_surr) {
  switch (id) {
    case ENV_QUADROTOR: return 2;
    case ENV_CARTPOLE: return 4;
    default: return 1;
  }
}

// s: one state row (float32). Writes done, violation, h[C].
__device__ inline void env_constraints_row(const EnvParams& ep, const float* s, bool& done, bool& viol, float* h) {
  if (ep.id == ENV_POINT_ROBOT) {
    // src/env/point_robot.py:96-131
    const double x = s[0], y = s[1];
    const double hx[2] = {0.4, -0.4}, hy[2] = {-1.2, 1.2};
    double md = __longlong_as_double(0x7ff0000000000000LL);   // +inf
    for (int k = 0; k < 2; ++k) {
      const double dx = hx[k] - x, dy = hy[k] - y;
      const double d = sqrt(dx * dx + dy * dy);
      md = fmin(d, md);
    }
    const double hv = 0.8 - md;
    h[0] = (float)hv;
    viol = hv > 0.0;
    const bool oob = (s[0] < -3.0f) || (s[0] > 3.0f) || (s[1] < -3.0f) || (s[1] > 3.0f);
    const double gx = x - 2.2, gy = y - 2.2;
    done = oob || (sqrt(gx * gx + gy * gy) <= 0.3);
  } else if (ep.id == ENV_QUADROTOR) {
    // src/env/quadrotor/quadrotor.py:83-158 with BoundedConstraint z in [0.5, 1.5]
    const double z = s[2];
    const double h0 = -z - (-0.5), h1 = z - 1.5;
    h[0] = (float)h0;
    h[1] = (float)h1;
    viol = (h0 > 0.0) || (h1 > 0.0);
    const float th = 1.48352986419518f;   // float32(85*pi/180)
    const float xt = (float)ep.thr0, zt = (float)ep.thr1;
    const bool oob = (s[0] < -xt) || (s[0] > xt) || (s[2] < -zt) || (s[2] > zt) || (s[4] < -th) || (s[4] > th);
    done = oob || viol;
  } else if (ep.id == ENV_CARTPOLE) {
    // src/env/poles/inverted_pendulum.py:11-26,79-121, constraints.py:216-247: BoundedConstraint
    // h = x @ F^T @ A^T - b in float64 with b = [x_thr, th_thr, x_thr, th_thr]
    const double x = s[0], t = s[1];
    const double hv[4] = {-x - ep.thr0, -t - ep.thr1, x - ep.thr0, t - ep.thr1};
    bool v = false;
    for (int k = 0; k < 4; ++k) {
      h[k] = (float)hv[k];
      v = v || (hv[k] > 0.0);
    }
    viol = v;
    done = v;
  } else {
    // ENV_TRACKING: src/env/tracking/pyth_veh3dofconti_surrcstr_data.py:253-338
    done = (fabsf(s[0]) > 5.f) || (fabsf(s[1]) > 2.f) || (fabsf(s[2]) > 3.14159274f);
    const float d = 1.4f;
    const float c = cosf(s[6]), sn = sinf(s[6]);
    float md = __int_as_float(0x7f800000);
    for (int v = 0; v < ep.n_surr; ++v) {
      const float* sv = s + ep.surr_start + 4 * v;
      const float xe = sv[0] * c + sv[1] * sn;
      const float ye = -sv[0] * sn + sv[1] * c;
      const float cp = cosf(sv[2]), sp = sinf(sv[2]);
      const float cx[2] = {xe + d * cp, xe - d * cp}, cy[2] = {ye + d * sp, ye - d * sp};
      const float ex[2] = {d, -d};
      for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) {
          const float dx = ex[i] - cx[j], dy = 0.f - cy[j];
          md = fminf(md, sqrtf(dx * dx + dy * dy));
        }
    }
    const double hv = 2.8284271247461903 - (double)md;
    h[0] = (float)hv;
    viol = hv > 0.0;
  }
}

}  // namespace drpo
