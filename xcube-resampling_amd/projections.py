"""Ellipsoidal map projections the engine supports, restated from PROJ.

The reference reaches these through pyproj/PROJ (``Transformer.from_crs``;
call sites reproject.py:124-126,347,398,483, rectify.py:196-203).  PROJ is
absent here, so the formulas PROJ uses are restated (radians in/out, unit
ellipsoid, ``a`` / false easting / northing applied by the caller exactly as
PROJ's ``pj_fwd`` / ``pj_inv`` do):

* ``TransverseMercator`` — PROJ ``tmerc`` with its default ``poder_engsager``
  algorithm (Krüger series to 6th order in n, Clenshaw summation: ``gatg``,
  ``clens``, ``clenS``), used for UTM zones (``+proj=utm``: k0 0.9996,
  central meridian 6*zone - 183, false easting 500 km, 10 000 km north offset
  for southern zones);
* ``LambertAzimuthalEqualArea`` — PROJ ``laea`` ellipsoidal oblique / equatorial
  / polar aspects (``pj_qsfn``, authalic latitude series ``pj_authset`` /
  ``pj_authlat``).

Parity: PROJ's results are not available here; the restatement is pinned by
the reference's own PROJ-dependent test goldens (tests/test_reproject.py,
tests/test_spatial.py, tests/test_rectify.py) that the GPU tests check.
All functions are vectorised numpy, float64.
"""

from __future__ import annotations

import math

import numpy as np

_ORDER = 6  # PROJ_ETMERC_ORDER


class Ellipsoid:
    def __init__(self, name: str, a: float, rf: float):
        self.name = name
        self.a = a
        self.rf = rf
        f = 1.0 / rf
        self.f = f
        self.es = 2.0 * f - f * f
        self.e = math.sqrt(self.es)
        self.one_es = 1.0 - self.es
        self.b = a * (1.0 - f)


WGS84 = Ellipsoid("WGS 84", 6378137.0, 298.257223563)
GRS80 = Ellipsoid("GRS 1980", 6378137.0, 298.257222101)


# ---- Clenshaw summations (PROJ tmerc.cpp) -----------------------------------
def _gatg(p, B, cos_2B, sin_2B):
    two_cos_2B = 2.0 * cos_2B
    h2 = 0.0
    h1 = p[-1]
    h = 0.0
    for coef in p[-2::-1]:
        h = -h2 + two_cos_2B * h1 + coef
        h2 = h1
        h1 = h
    return B + h * sin_2B


def _clens(a, arg_r):
    r = 2.0 * math.cos(arg_r)
    hr1 = 0.0
    hr = a[-1]
    for coef in a[-2::-1]:
        hr2 = hr1
        hr1 = hr
        hr = -hr2 + r * hr1 + coef
    return math.sin(arg_r) * hr


def _clenS(a, sin_arg_r, cos_arg_r, sinh_arg_i, cosh_arg_i):
    r = 2.0 * cos_arg_r * cosh_arg_i
    i = -2.0 * sin_arg_r * sinh_arg_i
    hi1 = hr1 = hi = 0.0
    hr = a[-1]
    for coef in a[-2::-1]:
        hr2 = hr1
        hi2 = hi1
        hr1 = hr
        hi1 = hi
        hr = -hr2 + r * hr1 - i * hi1 + coef
        hi = -hi2 + i * hr1 + r * hi1
    r = sin_arg_r * cosh_arg_i
    i = cos_arg_r * sinh_arg_i
    return r * hr - i * hi, r * hi + i * hr


class TransverseMercator:
    """PROJ tmerc, algo poder_engsager (tmerc.cpp setup_exact / exact_e_fwd /
    exact_e_inv).  lam/phi in radians relative to the central meridian."""

    def __init__(self, ell: Ellipsoid, k0: float, phi0: float = 0.0):
        self.ell = ell
        es = ell.es
        f = es / (1.0 + math.sqrt(1.0 - es))
        n = f / (2.0 - f)
        np_ = n
        cgb = [0.0] * _ORDER
        cbg = [0.0] * _ORDER
        utg = [0.0] * _ORDER
        gtu = [0.0] * _ORDER
        cgb[0] = n * (2 + n * (-2 / 3.0 + n * (-2 + n * (116 / 45.0 + n * (26 / 45.0 + n * (-2854 / 675.0))))))
        cbg[0] = n * (-2 + n * (2 / 3.0 + n * (4 / 3.0 + n * (-82 / 45.0 + n * (32 / 45.0 + n * (4642 / 4725.0))))))
        np_ = n * n
        cgb[1] = np_ * (7 / 3.0 + n * (-8 / 5.0 + n * (-227 / 45.0 + n * (2704 / 315.0 + n * (2323 / 945.0)))))
        cbg[1] = np_ * (5 / 3.0 + n * (-16 / 15.0 + n * (-13 / 9.0 + n * (904 / 315.0 + n * (-1522 / 945.0)))))
        np_ *= n
        cgb[2] = np_ * (56 / 15.0 + n * (-136 / 35.0 + n * (-1262 / 105.0 + n * (73814 / 2835.0))))
        cbg[2] = np_ * (-26 / 15.0 + n * (34 / 21.0 + n * (8 / 5.0 + n * (-12686 / 2835.0))))
        np_ *= n
        cgb[3] = np_ * (4279 / 630.0 + n * (-332 / 35.0 + n * (-399572 / 14175.0)))
        cbg[3] = np_ * (1237 / 630.0 + n * (-12 / 5.0 + n * (-24832 / 14175.0)))
        np_ *= n
        cgb[4] = np_ * (4174 / 315.0 + n * (-144838 / 6237.0))
        cbg[4] = np_ * (-734 / 315.0 + n * (109598 / 31185.0))
        np_ *= n
        cgb[5] = np_ * (601676 / 22275.0)
        cbg[5] = np_ * (444337 / 155925.0)
        np_ = n * n
        self.Qn = k0 / (1 + n) * (1 + np_ * (1 / 4.0 + np_ * (1 / 64.0 + np_ / 256.0)))
        utg[0] = n * (-0.5 + n * (2 / 3.0 + n * (-37 / 96.0 + n * (1 / 360.0 + n * (81 / 512.0 + n * (-96199 / 604800.0))))))
        gtu[0] = n * (0.5 + n * (-2 / 3.0 + n * (5 / 16.0 + n * (41 / 180.0 + n * (-127 / 288.0 + n * (7891 / 37800.0))))))
        utg[1] = np_ * (-1 / 48.0 + n * (-1 / 15.0 + n * (437 / 1440.0 + n * (-46 / 105.0 + n * (1118711 / 3870720.0)))))
        gtu[1] = np_ * (13 / 48.0 + n * (-3 / 5.0 + n * (557 / 1440.0 + n * (281 / 630.0 + n * (-1983433 / 1935360.0)))))
        np_ *= n
        utg[2] = np_ * (-17 / 480.0 + n * (37 / 840.0 + n * (209 / 4480.0 + n * (-5569 / 90720.0))))
        gtu[2] = np_ * (61 / 240.0 + n * (-103 / 140.0 + n * (15061 / 26880.0 + n * (167603 / 181440.0))))
        np_ *= n
        utg[3] = np_ * (-4397 / 161280.0 + n * (11 / 504.0 + n * (830251 / 7257600.0)))
        gtu[3] = np_ * (49561 / 161280.0 + n * (-179 / 168.0 + n * (6601661 / 7257600.0)))
        np_ *= n
        utg[4] = np_ * (-4583 / 161280.0 + n * (108847 / 3991680.0))
        gtu[4] = np_ * (34729 / 80640.0 + n * (-3418889 / 1995840.0))
        np_ *= n
        utg[5] = np_ * (-20648693 / 638668800.0)
        gtu[5] = np_ * (212378941 / 319334400.0)
        self.cgb, self.cbg, self.utg, self.gtu = cgb, cbg, utg, gtu
        Z = _gatg(cbg, phi0, math.cos(2 * phi0), math.sin(2 * phi0))
        self.Zb = -self.Qn * (Z + _clens(gtu, 2 * Z))

    def forward(self, lam, phi):
        lam = np.asarray(lam, dtype=np.float64)
        phi = np.asarray(phi, dtype=np.float64)
        Cn = _gatg(self.cbg, phi, np.cos(2 * phi), np.sin(2 * phi))
        sin_Cn, cos_Cn = np.sin(Cn), np.cos(Cn)
        sin_Ce, cos_Ce = np.sin(lam), np.cos(lam)
        cos_Cn_cos_Ce = cos_Cn * cos_Ce
        Cn = np.arctan2(sin_Cn, cos_Cn_cos_Ce)
        inv_denom_tan_Ce = 1.0 / np.hypot(sin_Cn, cos_Cn_cos_Ce)
        tan_Ce = sin_Ce * cos_Cn * inv_denom_tan_Ce
        Ce = np.arcsinh(tan_Ce)
        two_inv_denom_tan_Ce = 2 * inv_denom_tan_Ce
        two_inv_denom_tan_Ce_square = two_inv_denom_tan_Ce * inv_denom_tan_Ce
        tmp_r = cos_Cn_cos_Ce * two_inv_denom_tan_Ce_square
        sin_arg_r = sin_Cn * tmp_r
        cos_arg_r = cos_Cn_cos_Ce * tmp_r - 1
        sinh_arg_i = tan_Ce * two_inv_denom_tan_Ce
        cosh_arg_i = two_inv_denom_tan_Ce_square - 1
        dCn, dCe = _clenS(self.gtu, sin_arg_r, cos_arg_r, sinh_arg_i, cosh_arg_i)
        Cn = Cn + dCn
        Ce = Ce + dCe
        ok = np.abs(Ce) <= 2.623395162778
        x = np.where(ok, self.Qn * Ce, np.inf)
        y = np.where(ok, self.Qn * Cn + self.Zb, np.inf)
        return x, y

    def inverse(self, x, y):
        x = np.asarray(x, dtype=np.float64)
        y = np.asarray(y, dtype=np.float64)
        Cn = (y - self.Zb) / self.Qn
        Ce = x / self.Qn
        ok = np.abs(Ce) <= 2.623395162778
        sin_arg_r = np.sin(2 * Cn)
        cos_arg_r = np.cos(2 * Cn)
        exp_2_Ce = np.exp(2 * Ce)
        half_inv_exp_2_Ce = 0.5 / exp_2_Ce
        sinh_arg_i = 0.5 * exp_2_Ce - half_inv_exp_2_Ce
        cosh_arg_i = 0.5 * exp_2_Ce + half_inv_exp_2_Ce
        dCn, dCe = _clenS(self.utg, sin_arg_r, cos_arg_r, sinh_arg_i, cosh_arg_i)
        Cn = Cn + dCn
        Ce = Ce + dCe
        sin_Cn, cos_Cn = np.sin(Cn), np.cos(Cn)
        sinhCe = np.sinh(Ce)
        Ce = np.arctan2(sinhCe, cos_Cn)
        modulus_Ce = np.hypot(sinhCe, cos_Cn)
        Cn = np.arctan2(sin_Cn, modulus_Ce)
        tmp = 2 * modulus_Ce / (sinhCe * sinhCe + 1)
        sin_2_Cn = sin_Cn * tmp
        cos_2_Cn = tmp * modulus_Ce - 1.0
        phi = _gatg(self.cgb, Cn, cos_2_Cn, sin_2_Cn)
        return np.where(ok, Ce, np.inf), np.where(ok, phi, np.inf)


# ---- Lambert azimuthal equal area (PROJ laea.cpp) ------------------------------
_EPS10 = 1.0e-10
_P00, _P01, _P02 = 0.33333333333333333333, 0.17222222222222222222, 0.10257936507936507937
_P10, _P11, _P20 = 0.06388888888888888888, 0.06640211640211640212, 0.01677689594356261023


def _qsfn(sinphi, e, one_es):
    con = e * sinphi
    div1 = 1.0 - con * con
    div2 = 1.0 + con
    return one_es * (sinphi / div1 - (0.5 / e) * np.log((1.0 - con) / div2))


class LambertAzimuthalEqualArea:
    """PROJ laea, ellipsoidal (e_forward / e_inverse)."""

    def __init__(self, ell: Ellipsoid, phi0: float):
        self.ell = ell
        self.phi0 = phi0
        e, es, one_es = ell.e, ell.es, ell.one_es
        t = abs(phi0)
        if abs(t - math.pi / 2) < _EPS10:
            self.mode = "npole" if phi0 >= 0 else "spole"
        elif abs(t) < _EPS10:
            self.mode = "equit"
        else:
            self.mode = "obliq"
        self.qp = float(_qsfn(1.0, e, one_es))
        self.mmf = 0.5 / (1.0 - es)
        t2 = es * es
        self.apa = (es * _P00 + t2 * _P01 + t2 * es * _P02, t2 * _P10 + t2 * es * _P11,
                    t2 * es * _P20)
        if self.mode in ("npole", "spole"):
            self.dd = 1.0
        elif self.mode == "equit":
            self.rq = math.sqrt(0.5 * self.qp)
            self.dd = 1.0 / self.rq
            self.xmf = 1.0
            self.ymf = 0.5 * self.qp
        else:
            self.rq = math.sqrt(0.5 * self.qp)
            sinphi = math.sin(phi0)
            self.sinb1 = float(_qsfn(sinphi, e, one_es)) / self.qp
            self.cosb1 = math.sqrt(1.0 - self.sinb1 * self.sinb1)
            self.dd = math.cos(phi0) / (math.sqrt(1.0 - es * sinphi * sinphi) * self.rq *
                                        self.cosb1)
            self.ymf = self.rq / self.dd
            self.xmf = self.rq * self.dd

    def _authlat(self, beta):
        t = beta + beta
        a = self.apa
        return beta + a[0] * np.sin(t) + a[1] * np.sin(t + t) + a[2] * np.sin(t + t + t)

    def forward(self, lam, phi):
        lam = np.asarray(lam, dtype=np.float64)
        phi = np.asarray(phi, dtype=np.float64)
        e, one_es = self.ell.e, self.ell.one_es
        coslam, sinlam, sinphi = np.cos(lam), np.sin(lam), np.sin(phi)
        q = _qsfn(sinphi, e, one_es)
        if self.mode in ("obliq", "equit"):
            sinb = q / self.qp
            cosb2 = 1.0 - sinb * sinb
            cosb = np.where(cosb2 > 0, np.sqrt(np.maximum(cosb2, 0.0)), 0.0)
            if self.mode == "obliq":
                b = 1.0 + self.sinb1 * sinb + self.cosb1 * cosb * coslam
            else:
                b = 1.0 + cosb * coslam
            bad = np.abs(b) < _EPS10
            b = np.sqrt(2.0 / np.where(bad, 1.0, b))
            if self.mode == "obliq":
                y = self.ymf * b * (self.cosb1 * sinb - self.sinb1 * cosb * coslam)
            else:
                y = b * sinb * self.ymf
            x = self.xmf * b * cosb * sinlam
            return np.where(bad, np.inf, x), np.where(bad, np.inf, y)
        q = self.qp - q if self.mode == "npole" else self.qp + q
        pos = q >= 1e-15
        b = np.sqrt(np.where(pos, q, 0.0))
        x = np.where(pos, b * sinlam, 0.0)
        y = np.where(pos, coslam * (b if self.phi0 < 0.0 else -b), 0.0)
        return x, y

    def inverse(self, x, y):
        x = np.asarray(x, dtype=np.float64)
        y = np.asarray(y, dtype=np.float64)
        if self.mode in ("obliq", "equit"):
            x = x / self.dd
            y = y * self.dd
            rho = np.hypot(x, y)
            small = rho < _EPS10
            rho_s = np.where(small, 1.0, rho)
            asin_arg = 0.5 * rho_s / self.rq
            bad = asin_arg > 1.0
            sCe = 2.0 * np.arcsin(np.minimum(asin_arg, 1.0))
            cCe = np.cos(sCe)
            sCe = np.sin(sCe)
            x = x * sCe
            if self.mode == "obliq":
                ab = cCe * self.sinb1 + y * sCe * self.cosb1 / rho_s
                y = rho_s * self.cosb1 * cCe - y * self.sinb1 * sCe
            else:
                ab = y * sCe / rho_s
                y = rho_s * cCe
            lam = np.arctan2(x, y)
            phi = self._authlat(np.arcsin(np.clip(ab, -1.0, 1.0)))
            lam = np.where(small, 0.0, lam)
            phi = np.where(small, self.phi0, phi)
            return np.where(bad, np.inf, lam), np.where(bad, np.inf, phi)
        if self.mode == "npole":
            y = -y
        q = x * x + y * y
        ab = 1.0 - q / self.qp
        if self.mode == "spole":
            ab = -ab
        lam = np.arctan2(x, y)
        phi = self._authlat(np.arcsin(np.clip(ab, -1.0, 1.0)))
        return lam, phi
