"""Privacy-preserving logistic regression (the reference's flagship "model").

Reference: lib/encoding/logistic_regression.go.
  * DP side (EncodeLogisticRegression[WithProofs], :46-215): standardise with
    global (or local) mean/std, augment with a column of ones, compute the
    polynomial-approximation coefficients of the log-loss per record
    (level 1: x*(2y-1); level j>=2: ypart * x^{(x)j}, ypart = y - y(-1)^j - 1),
    sum over records, scale by PrecisionApproxCoefficients, round to int64 and
    encrypt.  Packing: level j at offset sum_{i<j}(d+1)^(i+1) (== the
    reference's j*(d+1)^j for k<=2, :96-111).
  * Querier side (DecodeLogisticRegression :217, FindMinimumWeights :693):
    decrypt, unpack, rescale, gradient descent on the approximated loss with
    the exact reference Cost (including its level-accumulation quirk, :526)
    and Gradient (:564) — here vectorised O((d+1)^2) instead of re-enumerating
    cartesian products each iteration.

MI355X design: the per-record coefficient sums are one tall-skinny fp64
GEMM  X^T diag(w) X  over N records (K13) — the HIP MFMA kernel
``lr_moments`` in csrc/kernels/dx_lr.hip (v_mfma_f64_16x16x4f64) when the DP's
records live on a GPU; the CPU path uses torch float64 matmul.
"""
from __future__ import annotations

import math
import time

import torch

from .. import native as nt
from ..crypto import elgamal as eg
from ..query import LogisticRegressionParameters
from ..utils import timers
from ..utils.log import get_logger

log = get_logger("logreg")

TAYLOR_COEFFICIENTS = [-math.log(2), -0.5, -0.125, 0, 0.0052]
MIN_AREA_COEFFICIENTS = [-0.714761, -0.5, -0.0976419]
POLY_APPROX_COEFFICIENTS = MIN_AREA_COEFFICIENTS
NUM_DPS = 10


# ----------------------------------------------------------------------------- data utilities
def standardise_with(X: torch.Tensor, means, sds) -> torch.Tensor:
    m = torch.as_tensor(means, dtype=torch.float64, device=X.device)
    s = torch.as_tensor(sds, dtype=torch.float64, device=X.device)
    return (X - m) / s


def compute_means_sds(X: torch.Tensor):
    """population mean / std per column (montanaflynn/stats StandardDeviation)."""
    return X.mean(0), X.std(0, unbiased=False)


def standardise(X: torch.Tensor) -> torch.Tensor:
    m, s = compute_means_sds(X)
    return (X - m) / s


def standardise_with_train(X_test: torch.Tensor, X_train: torch.Tensor) -> torch.Tensor:
    """StandardiseWithTrain (logistic_regression.go:943-965): the test matrix
    standardised with the TRAINING matrix's column means and (population)
    standard deviations."""
    m, s = compute_means_sds(X_train.to(torch.float64))
    return (X_test.to(torch.float64) - m) / s


def normalize(X: torch.Tensor) -> torch.Tensor:
    """Normalize (:985): column-wise min-max scaling with the matrix's own range."""
    return normalize_with(X, X)


def normalize_with(X_test: torch.Tensor, X_train: torch.Tensor) -> torch.Tensor:
    """NormalizeWith (:990-1012): the test matrix min-max scaled with the
    training matrix's column minima and maxima."""
    tr = X_train.to(torch.float64)
    mn, mx = tr.min(0).values, tr.max(0).values
    return (X_test.to(torch.float64) - mn) / (mx - mn)


def partition_dataset(X: torch.Tensor, y: torch.Tensor, ratio: float, shuffle: bool = False, seed: int = 0):
    """PartitionDataset (:1389-1420): the first int(n * ratio) records (after an
    optional seeded shuffle) for training, the rest for testing.  -> (X_train,
    y_train, X_test, y_test).  The shuffle order comes from numpy's seeded
    generator, not Go's math/rand (parity of the order itself is unpinned; the
    split sizes and the no-shuffle split are the reference's)."""
    import numpy as np

    n = X.shape[0]
    n_train = int(float(n) * ratio)
    idx = np.arange(n)
    if shuffle:
        idx = np.random.RandomState(seed).permutation(n)
    tr = torch.as_tensor(idx[:n_train], dtype=torch.long, device=X.device)
    te = torch.as_tensor(idx[n_train:], dtype=torch.long, device=X.device)
    return X.index_select(0, tr), y.index_select(0, tr.to(y.device)), X.index_select(0, te), \
        y.index_select(0, te.to(y.device))


def augment(X: torch.Tensor) -> torch.Tensor:
    return torch.cat([torch.ones((X.shape[0], 1), dtype=X.dtype, device=X.device), X], dim=1)


def n_coeffs(d: int, k: int) -> int:
    return sum((d + 1) ** (j + 1) for j in range(k))


# ----------------------------------------------------------------------------- approximation coefficients
def approx_coefficients(Xa: torch.Tensor, y: torch.Tensor, k: int) -> list:
    """Aggregated (summed over records) approximation coefficients per level.

    Xa: [N, d+1] standardised+augmented float64; y: [N] in {0,1}.
    Level 1: sum_i (2y_i-1) x_i ; level j: sum_i ypart_j(y_i) * x_i^{(x)j}
    flattened in cartesian (row-major) order."""
    y = y.to(torch.float64)
    out = [Xa.T @ (2 * y - 1)]
    for j in range(2, k + 1):
        ypart = y - y * ((-1.0) ** j) - 1.0
        if j == 2:
            out.append(lr_moment_gemm(Xa, ypart).reshape(-1))
        elif j == 3:
            out.append(torch.einsum("n,na,nb,nc->abc", ypart, Xa, Xa, Xa).reshape(-1))
        else:
            raise NotImplementedError("k > 3 is not supported (the reference packing is only valid for k <= 2)")
    return out


def distinct_approx_coefficients(x, y: int, k: int) -> list:
    """ComputeDistinctApproxCoefficients (lib/encoding/logistic_regression.go:
    322-363) for ONE (augmented) record: level j holds the products over the
    multisets i_1 <= ... <= i_j of the record's entries, in lexicographic
    order, times the level's sign -- (2y - 1) for level 1, then the previous
    level's sign times ypart = y - y (-1)^(j+1) - 1.  The cartesian layout of
    ``approx_coefficients`` is the same values with every ordering repeated."""
    import itertools

    xs = [float(v) for v in x]
    sign = 2.0 * float(y) - 1.0
    out = []
    for j in range(1, k + 1):
        if j > 1:
            sign *= float(y) - float(y) * (-1.0) ** j - 1.0
        lvl = []
        for combo in itertools.combinations_with_replacement(range(len(xs)), j):
            prod = 1.0
            for i in combo:
                prod *= xs[i]
            lvl.append(prod * sign + 0.0)  # + 0.0: no negative zeros
        out.append(lvl)
    return out


def lr_moment_gemm(Xa: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """sum_i w_i x_i x_i^T (K13).  On GPU: the native fp64-MFMA kernel."""
    if Xa.is_cuda:
        return nt.lr_moments(Xa.contiguous(), w.contiguous())
    return (Xa * w[:, None]).T @ Xa


def round_precision(v: torch.Tensor, precision: float) -> torch.Tensor:
    """int64(math.Round(x * precision)) — Go rounds half away from zero."""
    x = v * precision
    return (torch.sign(x) * torch.floor(torch.abs(x) + 0.5)).to(torch.int64)


def encode_coefficients_int_many(Xs: list, ys: list, params: LogisticRegressionParameters):
    """``encode_coefficients_int`` of several DPs' records as one fused batch
    (one encoder launch per DP, one reduction, one rounding pass: the same
    values as DP by DP) -> [n_dp, n_coeffs] int64, or None when the batch
    does not fit the fused GPU encoder (the caller then encodes per DP)."""
    if not Xs or params.K > 2 or not (params.Means and params.StandardDeviations):
        return None
    d = Xs[0].shape[1] if Xs[0] is not None and Xs[0].dim() == 2 else -1
    if d < 1 or d + 1 >= 48 or any(X is None or not X.is_cuda or X.dim() != 2 or X.shape[1] != d or len(X) == 0
                                   for X in Xs):
        return None
    tot = nt.lr_encode_many([X.to(torch.float64).contiguous() for X in Xs], ys, params.Means,
                            params.StandardDeviations, 0.0, -1.0)
    D = d + 1
    lv = tot[:, D, :D] if params.K == 1 else torch.cat([tot[:, D, :D], tot[:, :D, :D].reshape(len(Xs), -1)], 1)
    return round_precision(lv, params.PrecisionApproxCoefficients)


def encode_coefficients_int(X: torch.Tensor, y: torch.Tensor, params: LogisticRegressionParameters) -> torch.Tensor:
    """The packed int64 vector the DP encrypts (before encryption)."""
    X = X.to(torch.float64)
    if X.is_cuda and params.K <= 2 and X.shape[1] + 1 < 48:
        # one fused pass over the records: standardise + augment + level 1 + level 2 (dx_lr_encode)
        if params.Means and params.StandardDeviations:
            m = torch.as_tensor(params.Means, dtype=torch.float64)
            s = torch.as_tensor(params.StandardDeviations, dtype=torch.float64)
        else:
            m, s = compute_means_sds(X)
        # level-2 weight ypart = y - y*(-1)^2 - 1 = 0*y - 1
        lvl1, lvl2 = nt.lr_encode(X.contiguous(), y, m, s, 0.0, -1.0)
        levels = [lvl1] if params.K == 1 else [lvl1, lvl2.reshape(-1)]
        return torch.cat([round_precision(lv, params.PrecisionApproxCoefficients) for lv in levels])
    if params.Means and params.StandardDeviations:
        Xs = standardise_with(X, params.Means, params.StandardDeviations)
    else:
        Xs = standardise(X)
    Xa = augment(Xs)
    levels = approx_coefficients(Xa, y, params.K)
    return torch.cat([round_precision(lv, params.PrecisionApproxCoefficients) for lv in levels])


def encode_logistic_regression(X, y, params: LogisticRegressionParameters, pk: eg.PublicKeyTable,
                               with_proofs: bool = False, ranges=None):
    from ..ops.encoding import _encrypt_with_proofs

    d = params.NbrFeatures
    n = n_coeffs(d, params.K)
    if X is None or len(X) == 0:
        vals = [0] * n
    else:
        vals = encode_coefficients_int(torch.as_tensor(X, device=pk.device), torch.as_tensor(y, device=pk.device),
                                       params).cpu().tolist()
        assert len(vals) == n, (len(vals), n)
    return _encrypt_with_proofs(pk, vals, with_proofs, ranges)


# ----------------------------------------------------------------------------- querier: gradient descent
def unpack(vals, d: int, k: int) -> list:
    out, off = [], 0
    for j in range(k):
        m = (d + 1) ** (j + 1)
        out.append(torch.tensor(vals[off: off + m], dtype=torch.float64))
        off += m
    return out


def cost(weights: torch.Tensor, approx: list, N: int, lam: float) -> float:
    """logistic_regression.go:526 Cost, replicated exactly (the running sum is
    multiplied by each level's polynomial coefficient in turn)."""
    k = len(approx)
    d = approx[0].numel() - 1
    c = 0.0
    w = weights
    outer = w
    for j in range(k):
        if j == 0:
            term = float((w * approx[0]).sum())
        else:
            outer = torch.einsum("...a,b->...ab", outer, w) if j >= 1 else w
            term = float((outer.reshape(-1) * approx[j]).sum())
        c += term
        c *= POLY_APPROX_COEFFICIENTS[j + 1]
    c = c / N - POLY_APPROX_COEFFICIENTS[0]
    reg = float((weights[1:d + 1] ** 2).sum())
    return c + (lam / (2 * N)) * reg


def gradient(weights: torch.Tensor, approx: list, N: int, lam: float) -> torch.Tensor:
    """logistic_regression.go:564 Gradient, closed form for k <= 3."""
    k = len(approx)
    d1 = approx[0].numel()
    g = POLY_APPROX_COEFFICIENTS[1] * approx[0].clone()
    if k >= 2:
        A2 = approx[1].reshape(d1, d1)
        g += POLY_APPROX_COEFFICIENTS[2] * ((A2 + A2.T) @ weights)
    if k >= 3:
        A3 = approx[2].reshape(d1, d1, d1)
        S = A3 + A3.permute(1, 0, 2) + A3.permute(1, 2, 0)
        g += POLY_APPROX_COEFFICIENTS[3] * torch.einsum("iab,a,b->i", S, weights, weights)
    g = g / N
    reg = (lam / N) * weights
    reg[0] = 0.0
    return g + reg


def find_minimum_weights(approx: list, initial_weights, N: int, lam: float, step: float, max_iter: int,
                         timeout_s: float = 180.0) -> list:
    """logistic_regression.go:693 FindMinimumWeights (k == 1 -> closed form :680)."""
    k = len(approx)
    if k == 1:
        return [float(-POLY_APPROX_COEFFICIENTS[1] * a / lam) for a in approx[0].tolist()]
    if k == 2:
        return _find_minimum_weights_k2(approx, initial_weights, N, lam, step, max_iter, timeout_s)
    w = torch.tensor(list(initial_weights), dtype=torch.float64)
    min_w = w.clone()
    t0 = time.time()
    for it in range(max_iter):
        c = cost(w, approx, N, lam)
        if c >= 0.0:
            min_w = w.clone()
        w = w - step * gradient(w, approx, N, lam)
        if time.time() - t0 > timeout_s - 2.0:
            break
    return min_w.tolist()


def _find_minimum_weights_k2(approx, initial_weights, N, lam, step, max_iter, timeout_s):
    """k = 2 fast path of FindMinimumWeights: Cost and Gradient reduce to one
    (d+1)x(d+1) mat-vec per iteration with S = A2 + A2^T (w^T A2 w = w^T S w / 2),
    in float64 on the host in native code (``dx_lr_gd_k2``: no GIL held, ~10x
    the numpy loop); same iteration, same quirky Cost accumulation and
    min-weights rule."""
    import numpy as np

    from .. import native as nt

    C0, C1, C2 = POLY_APPROX_COEFFICIENTS[0], POLY_APPROX_COEFFICIENTS[1], POLY_APPROX_COEFFICIENTS[2]
    a0 = approx[0].cpu().numpy().astype(np.float64)
    d1 = a0.shape[0]
    A2 = approx[1].cpu().numpy().astype(np.float64).reshape(d1, d1)
    S = A2 + A2.T
    w0 = np.asarray(list(initial_weights), dtype=np.float64)
    return nt.lr_gd_k2(a0, S, w0, N, lam, step, max_iter, (C0, C1, C2))


def find_minimum_weights_with_encryption(encrypted: list, secret: int, initial_weights, N: int, lam: float,
                                         step: float, max_iter: int, precision: float):
    """FindMinimumWeightsWithEncryption (:746-766): the client decrypts the
    encrypted approximation coefficients (one CipherVector per level, with
    negatives), rescales them by ``precision`` and runs FindMinimumWeights.
    -> (weights, approx coefficients as lists of floats)."""
    approx = []
    for cv in encrypted:
        vals = eg.decrypt_auto(secret, cv).cpu().to(torch.float64)
        approx.append(vals / precision)
    w = find_minimum_weights(approx, initial_weights, N, lam, step, max_iter)
    return w, [a.tolist() for a in approx]


def decode_logistic_regression_values(vals, params: LogisticRegressionParameters) -> list:
    with timers.timed("GradientDescent", sync=False):
        approx = [a / params.PrecisionApproxCoefficients for a in unpack(vals, params.NbrFeatures, params.K)]
        init = params.InitialWeights or [0.0] * (params.NbrFeatures + 1)
        return find_minimum_weights(approx, init, params.NbrRecords, params.Lambda, params.Step, params.MaxIterations)


# ----------------------------------------------------------------------------- prediction & metrics
def predict(X: torch.Tensor, weights, means=None, sds=None) -> torch.Tensor:
    X = X.to(torch.float64)
    if means is not None and sds is not None:
        X = standardise_with(X, means, sds)
    Xa = augment(X)
    w = torch.as_tensor(weights, dtype=torch.float64, device=X.device)
    return torch.sigmoid(Xa @ w)


def predict_in_clear(x, weights) -> float:
    """PredictInClear (:808-817): sigmoid(w0 + sum_i w_{i+1} x_i) for one record."""
    s_ = sum(float(w) * float(v) for w, v in zip(list(weights)[1:], x))
    return 1.0 / (1.0 + math.exp(-float(weights[0]) - s_))


def predict_encrypted(encrypted_data: eg.CipherVector, weights, secret: int, precision_weights: float,
                      precision_data: float) -> float:
    """Predict (:820-852) for ONE encrypted record (Enc(round(x_i *
    precision_data)) per feature): the weighted sum with integer weights
    round(w_{i+1} * precision_weights) is evaluated homomorphically (the
    reference adds the ciphertext |w| times; here one scalar multiplication
    per feature, negatives as r - |w|, and one K5 reduction), decrypted with
    negatives, rescaled, and the sigmoid taken with the clear bias w0."""
    from ..crypto import bn254 as bn

    wi = [int(round_precision(torch.tensor([float(w)], dtype=torch.float64), precision_weights)[0])
          for w in list(weights)[1:]]
    n = len(encrypted_data)
    if n != len(wi):
        raise ValueError(f"{n} encrypted features for {len(wi)} weights")
    dev = encrypted_data.device
    sc = bn.scalars_tensor([w % bn.R for w in wi], dev)
    prod = encrypted_data.mul_scalars(sc)
    tot = eg.CipherVector(nt.g1_sum(prod.K.view(n, 1, 24)), nt.g1_sum(prod.C.view(n, 1, 24)))
    bound = sum(abs(w) for w in wi) * int(precision_data * 1e3 + 1) + 1
    dot = int(eg.decrypt_auto(secret, tot, bound=min(bound, 1 << 20)).cpu()[0])
    val = dot / (precision_weights * precision_data)
    return 1.0 / (1.0 + math.exp(-float(weights[0]) - val))


def logistic_regression_cost(weights, X: torch.Tensor, y: torch.Tensor, N: int, lam: float) -> float:
    """LogisticRegressionCost (:769-794) on clear data, including the
    reference's regulariser precedence (lambda / 2 * N, not lambda / (2N);
    a test-only helper)."""
    w = torch.as_tensor(weights, dtype=torch.float64)
    s1 = X.to(torch.float64) @ w
    cost = float((torch.log1p(torch.exp(s1)) - y.to(torch.float64) * s1).sum())
    return cost + float((w * w).sum()) * (lam / 2 * float(N))


def logistic_regression_gradient(weights, X: torch.Tensor, y: torch.Tensor, N: int, lam: float) -> list:
    """LogisticRegressionGradient (:797-817) on clear data."""
    w = torch.as_tensor(weights, dtype=torch.float64)
    X = X.to(torch.float64)
    g = X.T @ (torch.sigmoid(X @ w) - y.to(torch.float64)) + (lam / float(N)) * w
    return g.tolist()


def predict_homomorphic(X: torch.Tensor, weights, pk: eg.PublicKeyTable, secret: int, precision: float = 1e2):
    """Score encrypted features (logistic_regression.go PredictHomomorphic): the
    linear term is evaluated homomorphically on Enc(round(x*precision)) with
    integer weights round(w*precision), decrypted, then the sigmoid applied."""
    from ..crypto import bn254 as bn

    Xa = augment(X.to(torch.float64))
    xi = round_precision(Xa.reshape(-1), precision)
    cv, _ = eg.encrypt_ints(pk, xi)
    wi = round_precision(torch.as_tensor(weights, dtype=torch.float64), precision)
    N, d1 = Xa.shape
    ws = [int(v) for v in wi.repeat(N).tolist()]
    sc = bn.scalars_tensor([v % bn.R for v in ws], pk.device)
    prod = cv.mul_scalars(sc)
    K = nt.g1_sum(prod.K.view(N, d1, 24).transpose(0, 1).contiguous())
    C = nt.g1_sum(prod.C.view(N, d1, 24).transpose(0, 1).contiguous())
    bound = int(abs(xi).max()) * int(abs(wi).max() + 1) * d1 + 1
    dots = eg.DecryptionTable(bound, pk.device).decrypt(secret, eg.CipherVector(K, C))
    return torch.sigmoid(dots.to(torch.float64) / (precision * precision))


def metrics(pred: torch.Tensor, y: torch.Tensor, threshold: float = 0.5) -> dict:
    """Accuracy / precision / recall / F-score / AUC (logistic_regression.go:1103-1164)."""
    y = y.to(torch.float64)
    yhat = (pred >= threshold).to(torch.float64)
    tp = float(((yhat == 1) & (y == 1)).sum())
    tn = float(((yhat == 0) & (y == 0)).sum())
    fp = float(((yhat == 1) & (y == 0)).sum())
    fn = float(((yhat == 0) & (y == 1)).sum())
    n = max(1.0, float(y.numel()))
    precision = tp / (tp + fp) if tp + fp else 0.0
    recall = tp / (tp + fn) if tp + fn else 0.0
    f = 2 * precision * recall / (precision + recall) if precision + recall else 0.0
    # AUC via the rank statistic
    order = torch.argsort(pred)
    ranks = torch.empty_like(pred)
    ranks[order] = torch.arange(1, pred.numel() + 1, dtype=pred.dtype, device=pred.device)
    npos, nneg = float((y == 1).sum()), float((y == 0).sum())
    auc = (float(ranks[y == 1].sum()) - npos * (npos + 1) / 2) / (npos * nneg) if npos and nneg else 0.0
    return {"accuracy": (tp + tn) / n, "precision": precision, "recall": recall, "fscore": f, "auc": auc}


def partition_for_dp(X: torch.Tensor, y: torch.Tensor, dp_index: int, n_dps: int = NUM_DPS):
    """Deterministic per-DP split (the reference slices by a character of the
    DP's ServerIdentity string, logistic_regression.go:1427-1448; here by index)."""
    n = X.shape[0]
    per = n // n_dps
    s = dp_index * per
    e = n if dp_index == n_dps - 1 else s + per
    return X[s:e], y[s:e]


def load_csv_dataset(path: str, label_col: int = 0, drop_cols=()):
    """Dataset loader: CSV with the label in column 0 (logistic_regression.go GetDataForDataProvider)."""
    import numpy as np

    data = np.loadtxt(path, delimiter=",")
    keep = [c for c in range(data.shape[1]) if c != label_col and c not in drop_cols]
    X = torch.tensor(data[:, keep], dtype=torch.float64)
    y = torch.tensor(data[:, label_col], dtype=torch.int64)
    return X, y
