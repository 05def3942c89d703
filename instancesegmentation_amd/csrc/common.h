// Device-side helpers shared by every libisg kernel (gfx950 / CDNA4, wave64).
//
// The central abstraction is the *virtual tensor*: a raw conv output plus the
// per-channel transform its consumer applies on load (BatchNorm forward +
// activation, or BatchNorm backward), split in up to ISG_MAX_SEGS channel
// segments so a consumer can read a torch.cat(...) without materialising it
// (segment.py:31, 331, 485, 494). Per-channel coefficients are derived from
// double-precision statistics once per workgroup into LDS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/isg.h"
#include "residual.h"

#define ISG_DEV __device__ __forceinline__
#define ISG_DEV_HOST __host__ __device__ inline

typedef float f32x4 __attribute__((ext_vector_type(4)));


// Global-address-space access through a generic pointer. Pointers that come out of LDS
// tables (or any memory the compiler cannot trace to a kernel argument) otherwise turn
// into flat_load/flat_store, which count on lgkmcnt as well as vmcnt: every later LDS
// wait then drains all outstanding global loads and the loads serialise.
typedef const float __attribute__((address_space(1)))* gcfloat_p;
typedef float __attribute__((address_space(1)))* gfloat_p;
ISG_DEV float gld(const float* p, int64_t i) { return ((gcfloat_p)p)[i]; }
typedef const double __attribute__((address_space(1)))* gcdouble_p;
ISG_DEV double gld_d(const double* p, int64_t i) { return ((gcdouble_p)p)[i]; }
ISG_DEV void gst(float* p, int64_t i, float v) { ((gfloat_p)p)[i] = v; }
typedef const f32x4 __attribute__((address_space(1)))* gcf32x4_p;
// 16-B global load of 4 consecutive floats at p[i..i+3] (p + i 16-B aligned)
ISG_DEV f32x4 gld4(const float* p, int64_t i) { return *(gcf32x4_p)((gcfloat_p)p + i); }
typedef f32x4 __attribute__((address_space(1)))* gf32x4_p;
// 16-B global store of 4 consecutive floats at p[i..i+3] (p + i 16-B aligned)
ISG_DEV void gst4(float* p, int64_t i, f32x4 v) { *(gf32x4_p)((gfloat_p)p + i) = v; }

// Cooperative global -> LDS copy of n floats, dst[i] = src[off(i)] (off(i) < 0: 0), with U
// loads of each thread in flight together. A rolled `for (i = tid; i < n; i += nthreads)`
// loop around a predicated load pays one full memory round trip per iteration (the
// compiler waits for each load before the next iteration's branch): 9-34 serial L2 round
// trips in the weight staging of tap_conv / kp_stem / sub2_dgrad.
template <int U, class F>
ISG_DEV void coop_gather(float* dst, int n, int tid, int nthreads, const float* src, F off) {
    for (int i0 = tid; i0 < n; i0 += U * nthreads) {
        float v[U];
        bool z[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * nthreads;
            const int o = i < n ? off(i) : -1;
            z[u] = o < 0;
            v[u] = ((gcfloat_p)src)[o < 0 ? 0 : o];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * nthreads;
            if (i < n) dst[i] = z[u] ? 0.f : v[u];
        }
    }
}

// ---- per-channel coefficient table (LDS) -------------------------------------
// BN_FWD : v = act((x - c0) * c1 + c2)          c0=mean  c1=gamma*rstd  c2=beta, c3=slope
// BN_BWD : v = c0*g + c1*(y - c2) + c3          (BatchNorm2d backward)
// PLAIN  : v = x
struct ChanCoef {
    float c0, c1, c2, c3;
};

// ---- replicated accumulators (ISG_STAT_REP copies, include/isg.h) ---------------------
// replica chosen by the workgroup; spreads same-address atomics over the copies
ISG_DEV int rep_of_block() {
    return (int)((blockIdx.x + 7u * blockIdx.y + 13u * blockIdx.z) % ISG_STAT_REP);
}
// pointer to this workgroup's replica of an accumulator of n values
ISG_DEV double* rep_ptr(double* base, int n) { return base + (int64_t)rep_of_block() * n; }
// sum over replicas of element i of an accumulator of n values (fixed order)
ISG_DEV double rep_sum(const double* base, int n, int i) {
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < ISG_STAT_REP; ++r) s += base[(int64_t)r * n + i];
    return s;
}

// The fp64 coefficient math from replica-summed statistics: the one definition shared by
// fwd_coef / bwd_coef and the branch-free staging path (stage.h coef_issue / coef_finish),
// so every consumer derives bit-identical coefficients.
ISG_DEV void mean_rstd_of(double sum, double sumsq, float count, float eps, double& mean,
                          double& rstd) {
    double inv = 1.0 / (double)count;
    mean = sum * inv;
    double var = sumsq * inv - mean * mean;
    if (var < 0.0) var = 0.0;
    rstd = 1.0 / sqrt(var + (double)eps);
}
ISG_DEV ChanCoef fwd_coef_of(double mean, double rstd, float gamma, float beta, float slope) {
    ChanCoef k;
    k.c0 = (float)mean;
    k.c1 = (float)((double)gamma * rstd);
    k.c2 = beta;
    k.c3 = slope;
    return k;
}
ISG_DEV ChanCoef bwd_coef_of(double mean, double rstd, float gamma, double gs, double gxs,
                             float count) {
    const double gam = (double)gamma;
    const double inv = 1.0 / (double)count;
    const double mg = gs * inv;
    const double mgx = rstd * gxs * inv;  // mean(g * xhat); gxs = sum g*(y - mean), centred
    ChanCoef k;
    k.c0 = (float)(gam * rstd);
    k.c1 = (float)(-gam * rstd * rstd * mgx);
    k.c2 = (float)mean;
    k.c3 = (float)(-gam * rstd * mg);
    return k;
}

ISG_DEV void bn_mean_rstd(const isg_bn& bn, int c, double& mean, double& rstd) {
    if (bn.train) {
        mean_rstd_of(rep_sum(bn.stats, 4 * bn.C, c), rep_sum(bn.stats, 4 * bn.C, bn.C + c),
                     bn.count, bn.eps, mean, rstd);
    } else {
        mean = (double)bn.running_mean[c];
        rstd = 1.0 / sqrt((double)bn.running_var[c] + (double)bn.eps);
    }
}

// forward coefficients of a BN_FWD segment channel
ISG_DEV ChanCoef fwd_coef(const isg_bn& bn, const float* slope, int c) {
    if (bn.coef) {  // finalised once per layer (isg_bn_finalize)
        const f32x4 f = reinterpret_cast<const f32x4*>(bn.coef)[c];
        return ChanCoef{f[0], f[1], f[2], slope ? slope[c] : 0.f};
    }
    double mean, rstd;
    bn_mean_rstd(bn, c, mean, rstd);
    return fwd_coef_of(mean, rstd, bn.gamma[c], bn.beta[c], slope ? slope[c] : 0.f);
}

// backward coefficients: dy = A*g + B*(y-mean) + C
ISG_DEV ChanCoef bwd_coef(const isg_bn& bn, int c) {
    if (bn.coef) {
        const f32x4 f = reinterpret_cast<const f32x4*>(bn.coef)[bn.C + c];
        return ChanCoef{f[0], f[1], f[2], f[3]};
    }
    double mean, rstd;
    bn_mean_rstd(bn, c, mean, rstd);
    double gam = (double)bn.gamma[c];
    ChanCoef k;
    if (bn.train) {
        k = bwd_coef_of(mean, rstd, bn.gamma[c], rep_sum(bn.stats, 4 * bn.C, 2 * bn.C + c),
                        rep_sum(bn.stats, 4 * bn.C, 3 * bn.C + c), bn.count);
    } else {
        k.c0 = (float)(gam * rstd);
        k.c1 = 0.f;
        k.c2 = (float)mean;
        k.c3 = 0.f;
    }
    return k;
}

// A keypoint coordinate made safe for the reference's int() window bounds
// (train_instance.py:52-58): false for NaN / infinity (the reference's int() raises; the
// part is treated as not visible), else v clamped to [-(r + 2), extent + r + 2], which
// leaves the window [max(0,int(v-r)), min(extent-1,int(v+r+1))) unchanged — empty
// beyond those bounds either way — while keeping the int conversions defined.
ISG_DEV bool kp_coord(double& v, double r, int extent) {
    if (!(v == v) || v - v != 0.0) return false;
    const double lo = -(r + 2.0), hi = (double)extent + r + 2.0;
    v = v < lo ? lo : (v > hi ? hi : v);
    return true;
}

ISG_DEV float apply_act(float v, int act, float slope) {
    if (act == ISG_ACT_RELU) return v > 0.f ? v : 0.f;
    if (act == ISG_ACT_PRELU) return v > 0.f ? v : v * slope;  // torch prelu: x>0 ? x : w*x
    return v;
}

// Fill coefficient table for every channel of a vtensor (cooperatively by the block).
// Returns nothing; caller __syncthreads() afterwards.
ISG_DEV void load_vt_coefs(const isg_vtensor& vt, ChanCoef* coef, int tid, int nthreads) {
    int cbeg = 0;
    for (int s = 0; s < vt.nseg; ++s) {
        const isg_vseg& sg = vt.s[s];
        for (int c = tid; c < sg.C; c += nthreads) {
            ChanCoef k = {0.f, 1.f, 0.f, 0.f};
            if (sg.xform == ISG_XF_BN_FWD) {
                if (sg.bn.stats || !sg.bn.train) {
                    k = fwd_coef(sg.bn, sg.slope, c);
                } else {  // activation only, no BN
                    k.c0 = 0.f; k.c1 = 1.f; k.c2 = 0.f;
                    k.c3 = sg.slope ? sg.slope[c] : 0.f;
                }
            } else if (sg.xform == ISG_XF_BN_BWD) {
                k = bwd_coef(sg.bn, c);
            }
            coef[cbeg + c] = k;
        }
        cbeg += sg.C;
    }
}

// Value of virtual tensor `vt` at (n, global channel c, flat pixel pix) — caller did
// bounds. Segment selection uses selects on constant indices of the kernel-argument
// struct (scalar loads): a runtime index into a register array would spill it to
// scratch (cdna_hip_programming.md §5.4 rule 20).
ISG_DEV float vt_load(const isg_vtensor& vt, const ChanCoef* coef, int n, int c, int64_t hw,
                      int64_t pix) {
    const float* p = vt.s[0].p;
    const float* y = vt.s[0].y;
    int64_t ns = vt.s[0].n_stride, yns = vt.s[0].y_n_stride;
    int cb = 0, xf = vt.s[0].xform, act = vt.s[0].act;
    const int c1 = vt.s[0].C, c2 = c1 + vt.s[1].C;
    if (vt.nseg > 1 && c >= c1) {
        p = vt.s[1].p; y = vt.s[1].y; ns = vt.s[1].n_stride; yns = vt.s[1].y_n_stride;
        cb = c1; xf = vt.s[1].xform; act = vt.s[1].act;
    }
    if (vt.nseg > 2 && c >= c2) {
        p = vt.s[2].p; y = vt.s[2].y; ns = vt.s[2].n_stride; yns = vt.s[2].y_n_stride;
        cb = c2; xf = vt.s[2].xform; act = vt.s[2].act;
    }
    const int cl = c - cb;
    const float x = p[(int64_t)n * ns + (int64_t)cl * hw + pix];
    if (xf == ISG_XF_PLAIN) return x;
    const ChanCoef k = coef[c];
    if (xf == ISG_XF_BN_FWD) {
        const float v = (x - k.c0) * k.c1 + k.c2;
        return apply_act(v, act, k.c3);
    }
    const float yv = y[(int64_t)n * yns + (int64_t)cl * hw + pix];
    return k.c0 * x + k.c1 * (yv - k.c2) + k.c3;
}

// ---- reductions ----------------------------------------------------------------
ISG_DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
ISG_DEV double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ---- sinks ----------------------------------------------------------------------
struct SinkCoef {  // forward BN coefficients of an ACTBWD sink channel
    float mean, scale, beta, slope;
};

ISG_DEV void load_sink_coefs(const isg_sinks& sk, SinkCoef* sc, int tid, int nthreads) {
    for (int s = 0; s < sk.nsink; ++s) {
        const isg_sink& k = sk.s[s];
        if (k.mode != ISG_SINK_ACTBWD) continue;
        for (int c = tid; c < k.C; c += nthreads) {
            SinkCoef v = {0.f, 1.f, 0.f, 0.f};
            if (k.bn.stats || !k.bn.train) {
                ChanCoef f = fwd_coef(k.bn, k.slope, c);
                v.mean = f.c0; v.scale = f.c1; v.beta = f.c2;
            }
            v.slope = k.slope ? k.slope[c] : 0.f;
            sc[k.c0 + c] = v;
        }
    }
}

// Per-element sink application. Returns values to be reduced:
//   STORE : r0 = value (for sum), r1 = value^2
//   ACTBWD: r0 = g, r1 = g*(y - mean), r2 = prelu slope grad contribution
struct SinkRed {
    float r0, r1, r2;
};

ISG_DEV SinkRed sink_apply(const isg_sink& k, const SinkCoef* sc, int cglob, int n,
                           int64_t hw, int64_t pix, float v) {
    SinkRed r = {0.f, 0.f, 0.f};
    if (k.mode == ISG_SINK_NONE) return r;
    int cl = cglob - k.c0;
    int64_t off = (int64_t)n * k.n_stride + (int64_t)cl * hw + pix;
    if (k.mode == ISG_SINK_STORE) {
        if (k.bias) v += k.bias[cl];
        k.p[off] = v;
        r.r0 = v;
        r.r1 = v * v;
    } else if (k.mode == ISG_SINK_ACCUM) {
        k.p[off] += v;
        r.r0 = v;  // per-channel sums for a bias gradient (when stats is set)
        r.r1 = v * v;
    } else {
        float y = k.y[(int64_t)n * k.y_n_stride + (int64_t)cl * hw + pix];
        SinkCoef f = sc[cglob];
        float z = (y - f.mean) * f.scale + f.beta;  // BN output (pre-activation)
        float g = v;
        if (k.act == ISG_ACT_RELU) {
            g = z > 0.f ? v : 0.f;
        } else if (k.act == ISG_ACT_PRELU) {
            g = z > 0.f ? v : v * f.slope;
            r.r2 = z > 0.f ? 0.f : z * v;
        }
        k.p[off] = g;
        r.r0 = g;
        r.r1 = g * (y - f.mean);  // centred: no cancellation against mean*sum(g)
    }
    return r;
}

// which sink owns global channel c
ISG_DEV int sink_of(const isg_sinks& sk, int c) {
    int s = 0;
    if (sk.nsink > 1 && c >= sk.s[1].c0) s = 1;
    if (sk.nsink > 2 && c >= sk.s[2].c0) s = 2;
    return s;
}

// Block-level flush of per-channel partial reductions held in LDS (float) to the
// sink's double accumulators.
ISG_DEV void flush_sink_red(const isg_sinks& sk, const float* red0, const float* red1,
                            const float* red2, int Ctot, int tid, int nthreads) {
    for (int c = tid; c < Ctot; c += nthreads) {
        int s = sink_of(sk, c);
        const isg_sink& k = sk.s[s];
        int cl = c - k.c0;
        if (k.mode == ISG_SINK_STORE || k.mode == ISG_SINK_ACCUM) {
            if (k.stats) {
                double* st = rep_ptr(k.stats, 4 * k.C);
                atomicAdd(&st[cl], (double)red0[c]);
                atomicAdd(&st[k.C + cl], (double)red1[c]);
            }
        } else if (k.mode == ISG_SINK_ACTBWD) {
            if (k.bn.stats) {
                double* st = rep_ptr(k.bn.stats, 4 * k.C);
                atomicAdd(&st[2 * k.C + cl], (double)red0[c]);
                atomicAdd(&st[3 * k.C + cl], (double)red1[c]);
            }
            if (k.slope_grad && k.act == ISG_ACT_PRELU)
                atomicAdd(&rep_ptr(k.slope_grad, k.C)[cl], (double)red2[c]);
        }
    }
}

ISG_DEV bool sinks_need_red(const isg_sinks& sk) {
    for (int s = 0; s < sk.nsink; ++s) {
        if ((sk.s[s].mode == ISG_SINK_STORE || sk.s[s].mode == ISG_SINK_ACCUM) && sk.s[s].stats)
            return true;
        if (sk.s[s].mode == ISG_SINK_ACTBWD) return true;
    }
    return false;
}

// ---- diagnostic stamps (built only into the tools/kbench harness library) -------------
// STAMP(i): thread 0 of each workgroup records s_memrealtime (100 MHz, chip-global) in
// slot i of its 8-slot record. Compiled out of libisg.so.
#ifdef ISG_STAMPS
#define ISG_STAMP_MAXBLK 65536
// one buffer per translation unit (no relocatable device code); each .hip exposes it
// through isg_dbg_stamps_<file>() in the stamp build
static __device__ unsigned long long isg_stamps[ISG_STAMP_MAXBLK * 8];
#define ISG_STAMP_ACCESSOR(name)                                          \
    extern "C" void* name(void) {                                          \
        void* p = nullptr;                                                 \
        (void)hipGetSymbolAddress(&p, HIP_SYMBOL(isg_stamps));             \
        return p;                                                          \
    }
#define STAMP(i)                                                                          \
    do {                                                                                  \
        if (threadIdx.x == 0) {                                                           \
            const unsigned b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z); \
            if (b < ISG_STAMP_MAXBLK) isg_stamps[b * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                                 \
    } while (0)
#else
#define STAMP(i) do {} while (0)
#define ISG_STAMP_ACCESSOR(name)
#endif

// ---- error plumbing (host) -----------------------------------------------------
int32_t isg_set_error(int32_t code, const char* fmt, ...);
int32_t isg_check_launch(const char* what);
