"""Density evolution for (lambda, rho) ensembles.

* BEC: x_{l+1} = eps * lambda(1 - rho(1 - x_l)) -- for lambda = x^(dv-1),
  rho = x^(dc-1) this is tools/density_evolution.py:9-16 and the bisection of
  test_de_threshold.py:17-28 (pinned against their values in tests/golden).
* BI-AWGN: Gaussian approximation (Chung, Richardson, Urbanke, IEEE T-IT 2001):
  messages ~ N(mu, 2 mu); check update through phi(mu) = 1 - E[tanh(u/2)].
Host-side analysis tooling (numpy/scipy), used to choose and validate the
config-4 ensemble; not on the decoding path.
"""
import numpy as np

from .ensembles import Ensemble

# --------------------------------------------------------------------- BEC


def bec_de(ens, eps, iterations, threshold=0.0):
    """Erasure probability of v->c messages per iteration (starts with eps), in the
    output convention of tools/density_evolution.py:9-16 (values <= threshold dropped)."""
    out = [eps]
    x = eps
    for _ in range(iterations):
        nx = eps * ens.lam_poly(1.0 - ens.rho_poly(1.0 - x))
        if nx > threshold:
            out.append(nx)
            x = nx
        else:
            x = out[-1]
    return out


def bec_threshold(ens, iterations=100000, tol=1e-9, tolerance=1e-6):
    """Largest eps whose DE falls below `tolerance` (bisection as test_de_threshold.py:55-66)."""
    lo, hi = 0.0, 1.0
    while hi - lo > tol:
        mid = 0.5 * (lo + hi)
        x = 1.0
        ok = False
        for _ in range(iterations):
            x = mid * ens.lam_poly(1.0 - ens.rho_poly(1.0 - x))
            if x < tolerance:
                ok = True
                break
            # stationary above tolerance: a fixed point, stop early
        if ok:
            lo = mid
        else:
            hi = mid
    return 0.5 * (lo + hi)


# --------------------------------------------------------------- BI-AWGN GA
_GH_X, _GH_W = np.polynomial.hermite.hermgauss(80)


def phi(mu):
    """1 - E[tanh(u/2)], u ~ N(mu, 2 mu) (mu > 0), by Gauss-Hermite quadrature;
    the closed-form tail approximation of Chung et al. for large mu."""
    mu = np.atleast_1d(np.asarray(mu, dtype=np.float64))
    out = np.empty_like(mu)
    big = mu > 10.0
    out[big] = np.sqrt(np.pi / mu[big]) * np.exp(-mu[big] / 4.0) * (1.0 - 10.0 / (7.0 * mu[big]))
    m = mu[~big]
    if m.size:
        u = m[:, None] + 2.0 * np.sqrt(m[:, None]) * _GH_X[None, :]  # sqrt(2 * var) * x, var = 2 mu
        out[~big] = 1.0 - (np.tanh(u / 2.0) * _GH_W[None, :]).sum(1) / np.sqrt(np.pi)
    return out


def phi_inv(y, lo=1e-10, hi=400.0):
    """Inverse of phi on (0, 1] by bisection in log space."""
    y = float(y)
    if y >= 1.0:
        return 0.0
    a, b = lo, hi
    for _ in range(64):
        c = np.sqrt(a * b)
        if phi(c)[0] > y:
            a = c
        else:
            b = c
    return np.sqrt(a * b)


def awgn_ga(ens, sigma, iterations=500, target=60.0):
    """True if the GA mean of check->variable messages grows past `target`
    (successful decoding) at noise std sigma."""
    mu0 = 2.0 / sigma ** 2
    mu_u = 0.0
    for _ in range(iterations):
        # variable -> check means, mixed over variable degrees
        s = 0.0
        for i, li in ens.lam.items():
            s += li * phi(mu0 + (i - 1) * mu_u)[0]
        mu_new = 0.0
        for j, rj in ens.rho.items():
            mu_new += rj * phi_inv(1.0 - (1.0 - s) ** (j - 1))
        if mu_new > target:
            return True
        if abs(mu_new - mu_u) < 1e-10:
            return False
        mu_u = mu_new
    return False


def awgn_threshold(ens, lo=0.3, hi=1.5, tol=1e-4):
    """GA noise threshold sigma* (bisection)."""
    while hi - lo > tol:
        mid = 0.5 * (lo + hi)
        if awgn_ga(ens, mid):
            lo = mid
        else:
            hi = mid
    return 0.5 * (lo + hi)


def sigma_to_ebn0_db(sigma, rate):
    return 10.0 * np.log10(1.0 / (2.0 * rate * sigma ** 2))


def regular(dv, dc):
    return Ensemble({dv: 1.0}, {dc: 1.0})


# ------------------------------------------------- finite-length scaling (BEC)


def scaling_threshold_y(eps_star, dv, dc, tol=1e-6):
    """Fixed point y of y = 1 - (1 - eps* y^(dv-1))^(dc-1) at the threshold, iterated from 1
    (finite_length_scaling_calculation.py:9-16)."""
    prev, y = 0.0, 1.0
    while abs(y - prev) > tol:
        prev = y
        y = 1.0 - (1.0 - eps_star * y ** (dv - 1)) ** (dc - 1)
    return y


def scaling_alpha(eps_star, dv, dc):
    """Scaling parameter alpha of the (dv, dc) ensemble on the BEC
    (finite_length_scaling_calculation.py:18-21)."""
    y = scaling_threshold_y(eps_star, dv, dc)
    x = eps_star * y ** (dv - 1)
    return eps_star * np.sqrt(((dv - 1) / dv) * (1.0 / x - 1.0 / y))


def scaling_fer(n, eps, eps_star, alpha, beta=0.616949):
    """Waterfall block-error probability of the length-n ensemble under BP on BEC(eps):
    Q(sqrt(n) (eps* - beta n^(-2/3) - eps) / alpha) -- the law of
    finite_length_scaling_calculation.py:37-43 with the shift term of its :40 and the
    (3,6) shift beta = 0.616949 of tools/density_evolution.py:3-6."""
    from scipy.stats import norm
    z = np.sqrt(n) * (eps_star - beta * n ** (-2.0 / 3.0) - np.asarray(eps, dtype=np.float64))
    return norm.cdf(-z / alpha)
