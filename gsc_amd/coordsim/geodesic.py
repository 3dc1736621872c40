"""WGS-84 ellipsoidal distance (Vincenty inverse) used for link propagation delays.

The reference derives link delays from node coordinates with geopy's geodesic
distance (``coordsim/reader/reader.py:212-225``).  geopy is not installed, so
this module solves the inverse geodesic problem on the WGS-84 ellipsoid with
Vincenty's iteration (sub-millimetre agreement with Karney's algorithm for
non-antipodal points); link delays are rounded to integer milliseconds, so the
result is identical.
"""
import math

_A = 6378137.0
_F = 1 / 298.257223563
_B = (1 - _F) * _A


def distance_m(lat1: float, lon1: float, lat2: float, lon2: float) -> float:
    if lat1 == lat2 and lon1 == lon2:
        return 0.0
    L = math.radians(lon2 - lon1)
    U1 = math.atan((1 - _F) * math.tan(math.radians(lat1)))
    U2 = math.atan((1 - _F) * math.tan(math.radians(lat2)))
    sinU1, cosU1 = math.sin(U1), math.cos(U1)
    sinU2, cosU2 = math.sin(U2), math.cos(U2)
    lam = L
    for _ in range(200):
        sinLam, cosLam = math.sin(lam), math.cos(lam)
        sinSigma = math.hypot(cosU2 * sinLam, cosU1 * sinU2 - sinU1 * cosU2 * cosLam)
        if sinSigma == 0:
            return 0.0
        cosSigma = sinU1 * sinU2 + cosU1 * cosU2 * cosLam
        sigma = math.atan2(sinSigma, cosSigma)
        sinAlpha = cosU1 * cosU2 * sinLam / sinSigma
        cos2Alpha = 1 - sinAlpha * sinAlpha
        cos2SigmaM = cosSigma - 2 * sinU1 * sinU2 / cos2Alpha if cos2Alpha != 0 else 0.0
        C = _F / 16 * cos2Alpha * (4 + _F * (4 - 3 * cos2Alpha))
        lam_prev = lam
        lam = L + (1 - C) * _F * sinAlpha * (
            sigma + C * sinSigma * (cos2SigmaM + C * cosSigma * (-1 + 2 * cos2SigmaM ** 2)))
        if abs(lam - lam_prev) < 1e-12:
            break
    else:  # near-antipodal: fall back to a spherical estimate
        return _haversine(lat1, lon1, lat2, lon2)
    u2 = cos2Alpha * (_A * _A - _B * _B) / (_B * _B)
    A = 1 + u2 / 16384 * (4096 + u2 * (-768 + u2 * (320 - 175 * u2)))
    B = u2 / 1024 * (256 + u2 * (-128 + u2 * (74 - 47 * u2)))
    dSigma = B * sinSigma * (cos2SigmaM + B / 4 * (
        cosSigma * (-1 + 2 * cos2SigmaM ** 2)
        - B / 6 * cos2SigmaM * (-3 + 4 * sinSigma ** 2) * (-3 + 4 * cos2SigmaM ** 2)))
    return _B * A * (sigma - dSigma)


def _haversine(lat1, lon1, lat2, lon2, r=6371008.8):
    p1, p2 = math.radians(lat1), math.radians(lat2)
    dp, dl = p2 - p1, math.radians(lon2 - lon1)
    h = math.sin(dp / 2) ** 2 + math.cos(p1) * math.cos(p2) * math.sin(dl / 2) ** 2
    return 2 * r * math.asin(math.sqrt(h))
