// xrs_proj.hpp — PROJ operations on the device (gfx950), shared by
// xrs_transform (coordinate tables) and the fused reprojection gather
// (xrs_reproject_proj).  Each step restates one PROJ operation exactly as
// xcube_resampling_amd/projections.py + crs.py do in numpy (same formulas, same
// operation order, -ffp-contract=off): web Mercator (merc_s, webmerc),
// transverse Mercator (tmerc poder_engsager: Clenshaw gatg / clenS) and
// Lambert azimuthal equal area (laea e_forward / e_inverse), around PROJ's
// pj_fwd / pj_inv (lam0 + adjlon, unit-ellipsoid scaling, false origin).
// The device libm differs from the host's in the last bit of some
// transcendentals, so results agree with the numpy restatement to a few ulps.
#pragma once

#include <cmath>

#include "xrs_common.hpp"

namespace xrs {
namespace proj {

constexpr double kDegToRad = 0.017453292519943296;   // crs._DEG_TO_RAD
constexpr double kPi = 3.141592653589793;

// ---- f64 log / atan2 for the projection pipelines ---------------------------------
// The classic fdlibm reductions and minimax coefficients (e_log.c, s_atan.c;
// within 1 ulp of the correctly rounded result, 2 ulp for atan2 through the
// pi - r fold), written without branches: the library's versions are ~1.6x
// longer and the transform is VALU-issue bound.  atan2 takes
// one division, not two (round 5: within 2 ulp of numpy's arctan2 on 12 M
// points including band edges; 2 % of the fused 2u gather).
// log(x) for x >= 1 (NaN and +inf pass through).
__device__ inline double log_ge1(double x) {
  constexpr double kLg1 = 6.666666666666735130e-01, kLg2 = 3.999999999940941908e-01,
                   kLg3 = 2.857142874366239149e-01, kLg4 = 2.222219843214978396e-01,
                   kLg5 = 1.818357216161805012e-01, kLg6 = 1.531383769920937332e-01,
                   kLg7 = 1.479819860511658591e-01;
  constexpr double kLn2Hi = 6.93147180369123816490e-01, kLn2Lo = 1.90821492927058770002e-10;
  int e;
  double m = frexp(x, &e);                  // x = m 2^e, m in [0.5, 1)
  const bool lo = m < 0.70710678118654752440;
  m = lo ? m + m : m;                       // m in [sqrt(1/2), sqrt(2))
  const double dk = (double)(lo ? e - 1 : e);
  const double f = m - 1.0;
  const double sv = f / (2.0 + f), z = sv * sv, w = z * z;
  const double t1 = w * (kLg2 + w * (kLg4 + w * kLg6));
  const double t2 = z * (kLg1 + w * (kLg3 + w * (kLg5 + w * kLg7)));
  const double hfsq = 0.5 * f * f;
  const double r = dk * kLn2Hi - ((hfsq - (sv * (hfsq + t2 + t1) + dk * kLn2Lo)) - f);
  return x < INFINITY ? r : x;
}

// atan2(y, x) (not for both arguments 0 or infinite: the pipelines turn
// such points into non-finite results anyway)
__device__ inline double atan2_pp(double y, double x) {
  constexpr double kAt[11] = {3.33333333333329318027e-01, -1.99999999998764832476e-01,
                              1.42857142725034663711e-01, -1.11111104054623557880e-01,
                              9.09088713343650656196e-02, -7.69187620504482999495e-02,
                              6.66107313738753120669e-02, -5.83357013379057348645e-02,
                              4.97687799461593236017e-02, -3.65315727442169155270e-02,
                              1.62858201153657823623e-02};
  const double ax = fabs(x), ay = fabs(y);
  const bool swap = ay > ax;
  // a = p / q in [0, 1] is never formed: the band is chosen on p against
  // q's multiples and the reduced argument is one quotient of p, q (fdlibm's
  // reductions are accurate on either side of a band edge)
  const double p = swap ? ax : ay, q = swap ? ay : ax;
  const bool r0 = p >= 0.4375 * q, r1 = p >= 0.6875 * q;      // atan(1/2), atan(1) bands
  const double num = r1 ? p - q : (r0 ? (p + p) - q : p);
  const double den = r1 ? p + q : (r0 ? (q + q) + p : q);
  const double t = num / den, z = t * t, w = z * z;
  const double s1 =
      z * (kAt[0] + w * (kAt[2] + w * (kAt[4] + w * (kAt[6] + w * (kAt[8] + w * kAt[10])))));
  const double s2 = w * (kAt[1] + w * (kAt[3] + w * (kAt[5] + w * (kAt[7] + w * kAt[9]))));
  const double hi = r1 ? 7.85398163397448278999e-01 : 4.63647609000806093515e-01;
  const double lo = r1 ? 3.06161699786838301793e-17 : 2.26987774529616870924e-17;
  double r = r0 ? hi - ((t * (s1 + s2) - lo) - t) : t - t * (s1 + s2);
  r = swap ? 1.57079632679489655800e+00 - (r - 6.12323399573676603587e-17) : r;
  r = x < 0.0 ? 3.1415926535897931160e+00 - (r - 1.2246467991473531772e-16) : r;
  return copysign(r, y);
}

// ---- PROJ helpers (projections.py) ---------------------------------------------
// Clenshaw summation for the Gaussian <-> geodetic latitude (tmerc.cpp gatg)
__device__ inline double gatg(const double* p, double B, double cos_2B, double sin_2B) {
  const double two_cos_2B = 2.0 * cos_2B;
  double h2 = 0.0, h1 = p[5], h = 0.0;
#pragma unroll
  for (int k = 4; k >= 0; --k) {
    h = -h2 + two_cos_2B * h1 + p[k];
    h2 = h1;
    h1 = h;
  }
  return B + h * sin_2B;
}

// complex Clenshaw summation (tmerc.cpp clenS)
__device__ inline void clenS(const double* a, double sin_arg_r, double cos_arg_r,
                             double sinh_arg_i, double cosh_arg_i, double& dr, double& di) {
  double r = 2.0 * cos_arg_r * cosh_arg_i;
  double i = -2.0 * sin_arg_r * sinh_arg_i;
  double hi1 = 0.0, hr1 = 0.0, hi = 0.0, hr = a[5];
#pragma unroll
  for (int k = 4; k >= 0; --k) {
    const double hr2 = hr1, hi2 = hi1;
    hr1 = hr;
    hi1 = hi;
    hr = -hr2 + r * hr1 - i * hi1 + a[k];
    hi = -hi2 + i * hr1 + r * hi1;
  }
  r = sin_arg_r * cosh_arg_i;
  i = cos_arg_r * sinh_arg_i;
  dr = r * hr - i * hi;
  di = r * hi + i * hr;
}

// tmerc_fwd from the sines and cosines of the Gaussian latitude Cn and the
// longitude (shared by tmerc_fwd and the LAEA -> tmerc pipeline below)
__device__ inline void tmerc_fwd_tail(const XrsProjStep& s, double sin_Cn, double cos_Cn,
                                      double sin_Ce, double cos_Ce, double& x, double& y) {
  const double* gtu = s.c + 18;
  const double cos_Cn_cos_Ce = cos_Cn * cos_Ce;
  double Cn = atan2_pp(sin_Cn, cos_Cn_cos_Ce);
  // |(sin_Cn, cos_Cn cos_Ce)| <= 1: no scaling needed; rsqrt (within an ulp)
  // instead of hypot's scaled sequence and a division
  const double inv_denom_tan_Ce = rsqrt(sin_Cn * sin_Cn + cos_Cn_cos_Ce * cos_Cn_cos_Ce);
  const double tan_Ce = sin_Ce * cos_Cn * inv_denom_tan_Ce;
  // asinh through log (|tan_Ce| < 7 here: no overflow guard needed; absolute
  // error ~1e-16, i.e. ~1e-9 m, where the library's asinh keeps relative
  // precision near 0 at 1.6x the instructions).  sqrt(tan_Ce^2 + 1) is
  // 1 / |(sin_Cn, cos_Cn cos_Ce)| = inv_denom_tan_Ce (sin^2 + cos^2 = 1 for
  // both pairs, to an ulp): no square root
  double Ce = copysign(log_ge1(fabs(tan_Ce) + inv_denom_tan_Ce), tan_Ce);
  const double two_inv_denom_tan_Ce = 2 * inv_denom_tan_Ce;
  const double two_inv_denom_tan_Ce_square = two_inv_denom_tan_Ce * inv_denom_tan_Ce;
  const double tmp_r = cos_Cn_cos_Ce * two_inv_denom_tan_Ce_square;
  const double sin_arg_r = sin_Cn * tmp_r;
  const double cos_arg_r = cos_Cn_cos_Ce * tmp_r - 1;
  const double sinh_arg_i = tan_Ce * two_inv_denom_tan_Ce;
  const double cosh_arg_i = two_inv_denom_tan_Ce_square - 1;
  double dCn, dCe;
  clenS(gtu, sin_arg_r, cos_arg_r, sinh_arg_i, cosh_arg_i, dCn, dCe);
  Cn = Cn + dCn;
  Ce = Ce + dCe;
  const bool ok = fabs(Ce) <= 2.623395162778;
  x = ok ? s.Qn * Ce : INFINITY;
  y = ok ? s.Qn * Cn + s.Zb : INFINITY;
}

__device__ inline void tmerc_fwd(const XrsProjStep& s, double lam, double phi, double& x,
                                 double& y) {
  const double* cbg = s.c + 6;
  double s2p, c2p, sin_Cn, cos_Cn, sin_Ce, cos_Ce;
  sincos(2 * phi, &s2p, &c2p);
  const double Cn = gatg(cbg, phi, c2p, s2p);
  sincos(Cn, &sin_Cn, &cos_Cn);
  sincos(lam, &sin_Ce, &cos_Ce);
  tmerc_fwd_tail(s, sin_Cn, cos_Cn, sin_Ce, cos_Ce, x, y);
}

__device__ inline void tmerc_inv(const XrsProjStep& s, double x, double y, double& lam,
                                 double& phi) {
  const double* cgb = s.c;
  const double* utg = s.c + 12;
  double Cn = (y - s.Zb) / s.Qn;
  double Ce = x / s.Qn;
  const bool ok = fabs(Ce) <= 2.623395162778;
  double sin_arg_r, cos_arg_r;
  sincos(2 * Cn, &sin_arg_r, &cos_arg_r);
  const double exp_2_Ce = exp(2 * Ce);
  const double half_inv_exp_2_Ce = 0.5 / exp_2_Ce;
  const double sinh_arg_i = 0.5 * exp_2_Ce - half_inv_exp_2_Ce;
  const double cosh_arg_i = 0.5 * exp_2_Ce + half_inv_exp_2_Ce;
  double dCn, dCe;
  clenS(utg, sin_arg_r, cos_arg_r, sinh_arg_i, cosh_arg_i, dCn, dCe);
  Cn = Cn + dCn;
  Ce = Ce + dCe;
  double sin_Cn, cos_Cn;
  sincos(Cn, &sin_Cn, &cos_Cn);
  const double sinhCe = sinh(Ce);
  Ce = atan2(sinhCe, cos_Cn);
  const double modulus_Ce = hypot(sinhCe, cos_Cn);
  Cn = atan2(sin_Cn, modulus_Ce);
  const double tmp = 2 * modulus_Ce / (sinhCe * sinhCe + 1);
  const double sin_2_Cn = sin_Cn * tmp;
  const double cos_2_Cn = tmp * modulus_Ce - 1.0;
  const double ph = gatg(cgb, Cn, cos_2_Cn, sin_2_Cn);
  lam = ok ? Ce : INFINITY;
  phi = ok ? ph : INFINITY;
}

// laea modes (projections.py LambertAzimuthalEqualArea.mode)
constexpr int kNPole = 0, kSPole = 1, kEquit = 2, kObliq = 3;
constexpr double kEps10 = 1.0e-10;

__device__ inline double qsfn(double sinphi, double e, double one_es) {
  const double con = e * sinphi;
  const double div1 = 1.0 - con * con;
  const double div2 = 1.0 + con;
  return one_es * (sinphi / div1 - (0.5 / e) * log((1.0 - con) / div2));
}

// np.clip(v, -1, 1) (NaN stays NaN)
__device__ inline double clip1(double v) { return v < -1.0 ? -1.0 : (v > 1.0 ? 1.0 : v); }

__device__ inline double authlat(const XrsProjStep& s, double beta) {
  const double t = beta + beta;
  return beta + s.apa[0] * sin(t) + s.apa[1] * sin(t + t) + s.apa[2] * sin(t + t + t);
}

__device__ inline void laea_fwd(const XrsProjStep& s, double lam, double phi, double& x,
                                double& y) {
  double sinlam, coslam;
  sincos(lam, &sinlam, &coslam);
  const double sinphi = sin(phi);
  double q = qsfn(sinphi, s.e, s.one_es);
  if (s.mode == kObliq || s.mode == kEquit) {
    const double sinb = q / s.qp;
    const double cosb2 = 1.0 - sinb * sinb;
    const double cosb = cosb2 > 0 ? sqrt(fmax(cosb2, 0.0)) : 0.0;
    double b = s.mode == kObliq ? 1.0 + s.sinb1 * sinb + s.cosb1 * cosb * coslam
                                : 1.0 + cosb * coslam;
    const bool bad = fabs(b) < kEps10;
    b = sqrt(2.0 / (bad ? 1.0 : b));
    const double yy = s.mode == kObliq ? s.ymf * b * (s.cosb1 * sinb - s.sinb1 * cosb * coslam)
                                       : b * sinb * s.ymf;
    const double xx = s.xmf * b * cosb * sinlam;
    x = bad ? INFINITY : xx;
    y = bad ? INFINITY : yy;
    return;
  }
  q = s.mode == kNPole ? s.qp - q : s.qp + q;
  const bool pos = q >= 1e-15;
  const double b = sqrt(pos ? q : 0.0);
  x = pos ? b * sinlam : 0.0;
  y = pos ? coslam * (s.phi0 < 0.0 ? b : -b) : 0.0;
}

__device__ inline void laea_inv(const XrsProjStep& s, double x, double y, double& lam,
                                double& phi) {
  if (s.mode == kObliq || s.mode == kEquit) {
    x = x / s.dd;
    y = y * s.dd;
    const double rho = hypot(x, y);
    const bool small = rho < kEps10;
    const double rho_s = small ? 1.0 : rho;
    const double asin_arg = 0.5 * rho_s / s.rq;
    const bool bad = asin_arg > 1.0;
    double sCe, cCe;
    sincos(2.0 * asin(asin_arg > 1.0 ? 1.0 : asin_arg), &sCe, &cCe);   // np.minimum keeps NaN
    x = x * sCe;
    double ab;
    if (s.mode == kObliq) {
      ab = cCe * s.sinb1 + y * sCe * s.cosb1 / rho_s;
      y = rho_s * s.cosb1 * cCe - y * s.sinb1 * sCe;
    } else {
      ab = y * sCe / rho_s;
      y = rho_s * cCe;
    }
    double l = atan2(x, y);
    double p = authlat(s, asin(clip1(ab)));
    l = small ? 0.0 : l;
    p = small ? s.phi0 : p;
    lam = bad ? INFINITY : l;
    phi = bad ? INFINITY : p;
    return;
  }
  if (s.mode == kNPole) y = -y;
  const double q = x * x + y * y;
  double ab = 1.0 - q / s.qp;
  if (s.mode == kSPole) ab = -ab;
  lam = atan2(x, y);
  phi = authlat(s, asin(clip1(ab)));
}

// PROJ adjlon as crs._adjlon: wrap to [-pi, pi] when outside by more than 1e-12
__device__ inline double adjlon(double lam) {
  if (!(fabs(lam) >= kPi + 1e-12)) return lam;
  double w = lam + kPi;
  w = w - 2 * kPi * floor(w / (2 * kPi)) - kPi;
  return w;
}

// ---- LAEA inverse -> tmerc forward through sines and cosines --------------------
// The pipeline of a LAEA target grid over a UTM source (config 2u: EPSG:3035 ->
// EPSG:32632, reproject.py:472-496 per target pixel).  Every intermediate
// angle of apply_step<LAEA_INV> + apply_step<TMERC_FWD> is consumed only
// through its sine and cosine until tmerc's final atan2 / asinh, so they are
// carried as (sin, cos) pairs: 2 asin(a) by the double-angle identities,
// atan2(X, Y) as (X, Y) / hypot(X, Y), the longitude shift lam0_laea -
// lam0_tmerc and the latitude corrections of authlat (|d| < 0.003) and gatg
// (|d| < 0.004) as rotations (the small angles by Taylor terms to below an ulp).
// Ten f64 transcendentals per point (asin x2, sincos x5, atan2, ...) become
// two square roots, two hypots and two divisions; results agree with the
// two-step restatement to a few ulps (tests/test_transform_gpu.py tolerances),
// non-finite in the same places: the `small` / `bad` decisions are re-taken
// in the two-step order wherever the fast values are near a threshold.
struct LaeaTmerc {
  double sd, cd;     // sin / cos (lam0_laea - lam0_tmerc)
  double sp0, cp0;   // sin / cos phi0 (the LAEA centre, where rho < 1e-10)
  double inv_dd, half_inv_rq;   // 1 / dd and 0.5 / rq: products, not divisions, per point
};

__device__ inline LaeaTmerc laea_tmerc_setup(const XrsProjStep& s0, const XrsProjStep& s1) {
  LaeaTmerc k;
  sincos(s0.lam0 - s1.lam0, &k.sd, &k.cd);
  sincos(s0.phi0, &k.sp0, &k.cp0);
  k.inv_dd = 1.0 / s0.dd;
  k.half_inv_rq = 0.5 / s0.rq;
  return k;
}

// sin / cos of a small angle (|d| < 0.01): the dropped terms are < 1e-18
__device__ inline void sincos_small(double d, double& s, double& c) {
  const double d2 = d * d;
  s = d - d * d2 * (1.0 / 6.0) * (1.0 - d2 * (1.0 / 20.0));
  c = 1.0 - 0.5 * d2 * (1.0 - d2 * (1.0 / 12.0));
}

template <bool OBLIQ>
__device__ inline void laea_inv_tmerc_fwd(const XrsProjStep& s0, const XrsProjStep& s1,
                                          const LaeaTmerc& k, double& x, double& y) {
  // laea_inv's first half, with its two constant divisions as products by
  // reciprocals set up once per thread and the radius from sqrt / rsqrt of
  // one sum of squares (3 % and 1-2 % of the fused 2u gather,
  // profiles/r05_2u_int32_recip_ab.jsonl, r05_2u_rho_rsqrt_ab.jsonl).  Those
  // values are within 8 ulps of the two-step pipeline's xx, rho and a; the
  // `small` / `bad` DECISIONS are the two-step pipeline's own: wherever rho
  // or a lies within 2^-46 (relative, > 60 ulps) of its threshold they are
  // re-taken with laea_inv's operations (x / dd, hypot, 0.5 * rho / rq), so
  // a point never flips between data and fill (ADVICE r05;
  // tests/test_transform_gpu.py::test_fused_laea_tmerc_decisions_at_thresholds).
  double xx = (x - s0.x0) * s0.ra, yy = (y - s0.y0) * s0.ra;
  const double xx_in = xx;
  xx = xx * k.inv_dd;
  yy = yy * s0.dd;
  // |xx|, |yy| are a few earth radii at most: no scaling needed
  const double r2s = xx * xx + yy * yy;
  const double rho = sqrt(r2s);
  bool small = rho < kEps10;
  bool bad = (small ? 1.0 : rho) * k.half_inv_rq > 1.0;
  if (fabs(rho * k.half_inv_rq - 1.0) < 0x1p-46 || fabs(rho - kEps10) < 0x1p-46 * kEps10) {
    const double rx = hypot(xx_in / s0.dd, yy);   // laea_inv's x / dd, y * dd, hypot
    small = rx < kEps10;
    bad = 0.5 * (small ? 1.0 : rx) / s0.rq > 1.0;
  }
  const double rho_s = small ? 1.0 : rho;
  const double inv_rho_s = small ? 1.0 : rsqrt(r2s);
  const double a = rho_s * k.half_inv_rq;
  const double ac = a > 1.0 ? 1.0 : a;   // NaN stays NaN; a bad point's value is replaced
  const double ca = sqrt((1.0 - ac) * (1.0 + ac));
  const double sCe = 2.0 * ac * ca;             // sin (2 asin ac)
  const double cCe = 1.0 - 2.0 * ac * ac;       // cos (2 asin ac)
  const double X = xx * sCe;
  double ab, Y;
  if constexpr (OBLIQ) {
    ab = cCe * s0.sinb1 + yy * sCe * s0.cosb1 * inv_rho_s;
    Y = rho_s * s0.cosb1 * cCe - yy * s0.sinb1 * sCe;
  } else {
    ab = yy * sCe * inv_rho_s;
    Y = rho_s * cCe;
  }
  // longitude atan2(X, Y) (0 at the centre), shifted to tmerc's central meridian
  const double r2 = X * X + Y * Y;   // |X|, |Y| <= 2: no scaling needed
  const bool r0 = small || r2 == 0.0;
  const double ir = rsqrt(r0 ? 1.0 : r2);
  const double sl = r0 ? 0.0 : X * ir;
  const double cl = r0 ? ((small || !signbit(Y)) ? 1.0 : -1.0) : Y * ir;
  const double sin_Ce = sl * k.cd + cl * k.sd;
  const double cos_Ce = cl * k.cd - sl * k.sd;
  // latitude: beta = asin(clip(ab)), phi = authlat(beta) = beta + d
  const double sb = clip1(ab);
  const double cb = sqrt((1.0 - sb) * (1.0 + sb));
  const double s2b = 2.0 * sb * cb, c2b = (cb - sb) * (cb + sb);
  const double s4b = 2.0 * s2b * c2b, c4b = (c2b - s2b) * (c2b + s2b);
  const double s6b = s4b * c2b + c4b * s2b;
  double sd, cd;
  sincos_small(s0.apa[0] * s2b + s0.apa[1] * s4b + s0.apa[2] * s6b, sd, cd);
  const double sphi = small ? k.sp0 : sb * cd + cb * sd;
  const double cphi = small ? k.cp0 : cb * cd - sb * sd;
  // tmerc_fwd: Gaussian latitude Cn = phi + gatg correction
  const double s2p = 2.0 * sphi * cphi, c2p = (cphi - sphi) * (cphi + sphi);
  double sg, cg;
  sincos_small(gatg(s1.c + 6, 0.0, c2p, s2p), sg, cg);
  const double sin_Cn = sphi * cg + cphi * sg;
  const double cos_Cn = cphi * cg - sphi * sg;
  double px, py;
  tmerc_fwd_tail(s1, sin_Cn, cos_Cn, sin_Ce, cos_Ce, px, py);
  x = bad ? INFINITY : s1.a * px + s1.x0;
  y = bad ? INFINITY : s1.a * py + s1.y0;
}

// one pipeline step (crs._projection forward / inverse, webmerc_forward /
// _inverse); the kind is a template parameter, so a kernel holds only the code
// (and registers) of its own pipeline
template <int KIND>
__device__ inline void apply_step(const XrsProjStep& s, double& x, double& y) {
  const double rad_to_deg = 1.0 / kDegToRad;   // crs._RAD_TO_DEG_FACTOR
  if constexpr (KIND == XRS_PROJ_WEBMERC_FWD) {
    const double lam = x * kDegToRad, phi = y * kDegToRad;
    x = s.a * lam;
    y = s.a * asinh(tan(phi));
  } else if constexpr (KIND == XRS_PROJ_WEBMERC_INV) {
    const double lam = x * s.ra;
    const double phi = atan(sinh(y * s.ra));
    x = lam * rad_to_deg;
    y = phi * rad_to_deg;
  } else if constexpr (KIND == XRS_PROJ_TMERC_FWD || KIND == XRS_PROJ_LAEA_FWD) {
    const double lam = adjlon(x * kDegToRad - s.lam0);
    const double phi = y * kDegToRad;
    double px, py;
    if constexpr (KIND == XRS_PROJ_TMERC_FWD) tmerc_fwd(s, lam, phi, px, py);
    else laea_fwd(s, lam, phi, px, py);
    x = s.a * px + s.x0;
    y = s.a * py + s.y0;
  } else if constexpr (KIND == XRS_PROJ_TMERC_INV || KIND == XRS_PROJ_LAEA_INV) {
    const double xx = (x - s.x0) * s.ra, yy = (y - s.y0) * s.ra;
    double lam, phi;
    if constexpr (KIND == XRS_PROJ_TMERC_INV) tmerc_inv(s, xx, yy, lam, phi);
    else laea_inv(s, xx, yy, lam, phi);
    lam = adjlon(lam + s.lam0);
    x = lam * rad_to_deg;
    y = phi * rad_to_deg;
  }
}

// pipeline = step K0 then step K1 (0: none); FAST 1 / 2: the LAEA (oblique /
// equatorial) -> tmerc pair through laea_inv_tmerc_fwd (chosen on the host,
// fast_kind), with its per-thread constants set up once
constexpr int kFastNone = 0, kFastObliq = 1, kFastEquit = 2;

inline int fast_kind(int k0, int k1, const XrsProjStep& s0) {
  if (k0 != XRS_PROJ_LAEA_INV || k1 != XRS_PROJ_TMERC_FWD) return kFastNone;
  return s0.mode == kObliq ? kFastObliq : (s0.mode == kEquit ? kFastEquit : kFastNone);
}

template <int K0, int K1, int FAST>
struct Pipeline {
  LaeaTmerc k{};
  __device__ Pipeline(const XrsProjStep& s0, const XrsProjStep& s1) {
    if constexpr (FAST != kFastNone) k = laea_tmerc_setup(s0, s1);
  }
  __device__ void operator()(const XrsProjStep& s0, const XrsProjStep& s1, double& x,
                             double& y) const {
    if constexpr (FAST != kFastNone) {
      laea_inv_tmerc_fwd<FAST == kFastObliq>(s0, s1, k, x, y);
    } else {
      if constexpr (K0 != 0) apply_step<K0>(s0, x, y);
      if constexpr (K1 != 0) apply_step<K1>(s1, x, y);
    }
  }
};

}  // namespace proj
}  // namespace xrs
