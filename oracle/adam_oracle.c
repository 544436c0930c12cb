/*
 * TEST INFRASTRUCTURE — plain-C restatement of torch.optim.Adam's update (checker + CPU baseline).
 *
 * Restates the non-capturable single-tensor algorithm of torch/optim/adam.py:394-547 (the
 * reference delegates its Adam math there: zero1.py:88, zero2.py:120, zero3.py:161; pinned
 * torch==2.4.1 at pyproject.toml:13) in the rounding order of torch's CPU kernels:
 *   m = fmaf(1-b1, g-m, m)                 exp_avg.lerp_(grad, 1-b1)     (ATen Lerp.h, w < 0.5)
 *   v = fmaf((1-b2)*g, g, v*b2)            exp_avg_sq.mul_(b2).addcmul_(grad, grad, 1-b2)
 *   denom = sqrtf(v)/bc2_sqrt + eps        (exp_avg_sq.sqrt() / bias_correction2_sqrt).add_(eps)
 *   p = p + (neg_step*m)/denom             param.addcdiv_(exp_avg, denom, value=-step_size)
 * plus the ZeRO grad averaging (zero1.py:84 / zero2.py:111: grad /= ws) and the ZeRO-1 carry
 * A_t = (S + (ws-1)·A_{t-1})/ws.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library; the
 * product never does.  Build: oracle/Makefile → oracle/_build/libadam_oracle.so
 * (gcc -O2 -ffp-contract=off -fno-math-errno: sqrtf is the correctly rounded sqrtss).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct {
  float one_minus_beta1, beta2, one_minus_beta2, neg_step_size, bc2_sqrt, eps;
  float weight_decay, decay_mul, grad_div, carry_mul;
  int32_t amsgrad, maximize;
} oracle_hparams;

/* Scalars exactly as adam.py:508-537 derives them (python doubles, then fp32 at use). */
void oracle_hparams_init(double lr, double beta1, double beta2, double eps, double wd, int decoupled,
                         int amsgrad, int maximize, int64_t step, double grad_div,
                         double carry_mul, oracle_hparams* hp) {
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2 = 1.0 - pow(beta2, (double)step);
  hp->one_minus_beta1 = (float)(1.0 - beta1);
  hp->beta2 = (float)beta2;
  hp->one_minus_beta2 = (float)(1.0 - beta2);
  hp->neg_step_size = (float)(-(lr / bc1));
  hp->bc2_sqrt = (float)pow(bc2, 0.5);
  hp->eps = (float)eps;
  hp->weight_decay = decoupled ? 0.0f : (float)wd;
  hp->decay_mul = decoupled ? (float)(1.0 - lr * wd) : 1.0f;
  hp->grad_div = (float)grad_div;
  hp->carry_mul = (float)carry_mul;
  hp->amsgrad = amsgrad;
  hp->maximize = maximize;
}

static inline float adam_elem(float gsum, float* p, float* m, float* v, float* vmax, float* carry,
                              const oracle_hparams* hp) {
  float s = gsum;
  if (carry) s = s + hp->carry_mul * *carry;
  float g = s / hp->grad_div;
  if (carry) *carry = g;
  if (hp->maximize) g = -g;
  if (hp->weight_decay != 0.0f) g = fmaf(hp->weight_decay, *p, g);
  float pp = *p * hp->decay_mul;
  float mm = fmaf(hp->one_minus_beta1, g - *m, *m);
  float vv = fmaf(hp->one_minus_beta2 * g, g, *v * hp->beta2);
  float use = vv;
  if (hp->amsgrad) {
    *vmax = fmaxf(*vmax, vv);
    use = *vmax;
  }
  const float denom = sqrtf(use) / hp->bc2_sqrt + hp->eps;
  pp = pp + (hp->neg_step_size * mm) / denom;
  *p = pp;
  *m = mm;
  *v = vv;
  return pp;
}

static inline float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static inline uint16_t f32_to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

/* fp32 params/grads: p, m, v (and vmax/carry when non-NULL) updated in place. */
void oracle_adam_f32(float* p, const float* g, float* m, float* v, float* vmax, float* carry,
                     int64_t n, const oracle_hparams* hp) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i)
    adam_elem(g ? g[i] : 0.0f, &p[i], &m[i], &v[i], vmax ? &vmax[i] : 0, carry ? &carry[i] : 0, hp);
}

/* bf16 grads and params with an fp32 master: master/m/v updated, p_bf16 = bf16(master). */
void oracle_adam_bf16(float* master, uint16_t* p_bf16, const uint16_t* g, float* m, float* v,
                      float* vmax, float* carry, int64_t n, const oracle_hparams* hp) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const float pp = adam_elem(g ? bf16_to_f32(g[i]) : 0.0f, &master[i], &m[i], &v[i],
                               vmax ? &vmax[i] : 0, carry ? &carry[i] : 0, hp);
    if (p_bf16) p_bf16[i] = f32_to_bf16(pp);
  }
}

/* Split master (include/zero_amd.h ZS_BF16_SPLIT): the fp32 master's bits u are held as the bf16
 * param hi = RNE(u) and an int16 residual lo = u - (hi << 16); u = (hi << 16) + sext(lo).  The
 * residual +0x8000 (an exact tie rounded down to an even hi) does not fit int16 and is stored as
 * 0x7FFF: that master moves 1 ulp toward zero, hi is unchanged. */
static inline float join_master(uint16_t hi, uint16_t lo) {
  const uint32_t u = ((uint32_t)hi << 16) + (uint32_t)(int32_t)(int16_t)lo;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static inline uint16_t master_residual(float p, uint16_t hi) {
  uint32_t u;
  memcpy(&u, &p, 4);
  const uint32_t d = u - ((uint32_t)hi << 16);
  return d == 0x8000u ? (uint16_t)0x7fffu : (uint16_t)(d & 0xffffu);
}

/* bf16 grads and params with a split master: hi (the bf16 param) and lo updated in place. */
void oracle_adam_bf16_split(uint16_t* hi, uint16_t* lo, const uint16_t* g, float* m, float* v,
                            float* vmax, float* carry, int64_t n, const oracle_hparams* hp) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    float master = join_master(hi[i], lo[i]);
    const float pp = adam_elem(g ? bf16_to_f32(g[i]) : 0.0f, &master, &m[i], &v[i],
                               vmax ? &vmax[i] : 0, carry ? &carry[i] : 0, hp);
    hi[i] = f32_to_bf16(pp);
    lo[i] = master_residual(pp, hi[i]);
  }
}

/* The split-master encoding alone (tests: round trips and the tie rule). */
void oracle_split_master(const float* master, uint16_t* hi, uint16_t* lo, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    hi[i] = f32_to_bf16(master[i]);
    lo[i] = master_residual(master[i], hi[i]);
  }
}

void oracle_join_master(const uint16_t* hi, const uint16_t* lo, float* master, int64_t n) {
  for (int64_t i = 0; i < n; ++i) master[i] = join_master(hi[i], lo[i]);
}

int oracle_num_threads(void) {
#ifdef _OPENMP
  extern int omp_get_max_threads(void);
  return omp_get_max_threads();
#else
  return 1;
#endif
}
