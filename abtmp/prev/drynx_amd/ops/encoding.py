"""Data-provider encoders and querier decoders for every Drynx operation.

Reference: lib/encoding/encode_decode.go (dispatch, :14-254) and one file per
operation (sum.go, mean.go, variance.go, cosim.go, frequency_count.go,
min_max.go, OR_AND.go, set_union_intersection.go, linear_regression_dims.go,
model_evaluation.go, logistic_regression.go).

MI355X design: a DP's local statistics are exact int64 reductions over its
records on the party's device (K14 of SURVEY §2.3 — never fp MFMA for exact
integers), then every output of the response is encrypted by ONE batched
fixed-base ElGamal kernel launch (K2/K3) instead of one goroutine per
ciphertext.  With proofs, the (value, r) pairs are handed back as a
``RangeProofBatch`` so all range proofs of the response are produced by one
batched prover call.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from fractions import Fraction
from typing import Optional

import torch

from ..crypto import bn254 as bn
from ..crypto import elgamal as eg
from ..query import Operation


@dataclass
class CreateProofBatch:
    """Inputs of the range proofs of one response (lib/range CreateProof, batched).

    values[i], r[i] (scalars tensor row), cipher i of ``cv``; u[i], l[i], offset[i];
    sig_col[i] = which output column of the IV signatures proves value i."""
    values: list
    r: torch.Tensor
    cv: eg.CipherVector
    u: list
    l: list
    sig_col: list
    offset: list = field(default_factory=list)
    values_t: Optional[torch.Tensor] = None   # the values as a device int64 tensor (prover digits on the device)

    def __len__(self):
        return len(self.values)


def cat_proof_batches(batches: list) -> "CreateProofBatch":
    """One CreateProofBatch out of several (several DPs' responses)."""
    if len(batches) == 1:
        return batches[0]
    offs = []
    for b in batches:
        offs += list(b.offset) if b.offset else [0] * len(b)
    vt = torch.cat([b.values_t for b in batches]) if all(b.values_t is not None for b in batches) else None
    return CreateProofBatch([v for b in batches for v in b.values], torch.cat([b.r for b in batches]).contiguous(),
                            eg.CipherVector.cat([b.cv for b in batches]), [x for b in batches for x in b.u],
                            [x for b in batches for x in b.l], [x for b in batches for x in b.sig_col], offs, vt)


@dataclass
class EncodeResult:
    cv: eg.CipherVector
    clear: list
    proofs: Optional[CreateProofBatch] = None


def _ranges_uvl(ranges, n):
    """ranges[i] = [u, l] or [u, l, offset]."""
    us, ls, offs = [], [], []
    for i in range(n):
        rg = ranges[i]
        us.append(int(rg[0]))
        ls.append(int(rg[1]))
        offs.append(int(rg[2]) if len(rg) > 2 else 0)
    return us, ls, offs


def _encrypt_with_proofs(pk: eg.PublicKeyTable, values, with_proofs: bool, ranges, sig_cols=None):
    vals = [int(v) for v in values]
    cv, r = eg.encrypt_ints(pk, vals)
    prf = None
    if with_proofs:
        us, ls, offs = _ranges_uvl(ranges, len(vals))
        cols = list(range(len(vals))) if sig_cols is None else sig_cols
        prf = CreateProofBatch(vals, r, cv, us, ls, cols, offs)
    return EncodeResult(cv, vals, prf)


def _t(x, device):
    return x.to(device) if isinstance(x, torch.Tensor) else torch.tensor(x, dtype=torch.int64, device=device)


# ----------------------------------------------------------------------------- simple moments
def _moments(name: str, data, device, n_cols: int) -> list:
    """One DP's outputs of a moment operation through the K14 kernel (one
    launch, one copy of the few results to the host)."""
    cols = [_t(c, device).reshape(-1).to(torch.int64) for c in data[:n_cols]]
    Z = torch.stack(cols, dim=1)
    return batch_values(name, Z, [Z.shape[0]])[0].cpu().tolist()


def encode_sum(data, pk, with_proofs=False, ranges=None):
    """sum.go:17 — [sum x]."""
    return _encrypt_with_proofs(pk, _moments("sum", data, pk.device, 1), with_proofs, ranges)


def encode_mean(data, pk, with_proofs=False, ranges=None):
    """mean.go:17 — [sum x, N]."""
    return _encrypt_with_proofs(pk, _moments("mean", data, pk.device, 1), with_proofs, ranges)


def encode_variance(data, pk, with_proofs=False, ranges=None):
    """variance.go:17 — [sum x, N, sum x^2]."""
    return _encrypt_with_proofs(pk, _moments("variance", data, pk.device, 1), with_proofs, ranges)


def encode_cosim(data, pk, with_proofs=False, ranges=None):
    """cosim.go:18 — [sum a, sum b, sum a^2, sum b^2, sum ab]."""
    return _encrypt_with_proofs(pk, _moments("cosim", data, pk.device, 2), with_proofs, ranges)


def encode_frequency_count(data, qmin, qmax, pk, with_proofs=False, ranges=None):
    """frequency_count.go:18 — histogram over [qmin, qmax]."""
    x = _t(data[0], pk.device)
    n = qmax - qmin + 1
    mask = (x >= qmin) & (x <= qmax)
    hist = torch.bincount((x[mask] - qmin).to(torch.int64), minlength=n)[:n]
    return _encrypt_with_proofs(pk, hist.cpu().tolist(), with_proofs, ranges)


def encode_model_evaluation(data, pk, with_proofs=False, ranges=None):
    """model_evaluation.go:17 — [N, sum y, sum y^2, sum (pred - y)^2]; data = [y, pred]."""
    return _encrypt_with_proofs(pk, _moments("MLeval", data, pk.device, 2), with_proofs, ranges)


def encode_lin_reg(data, pk, with_proofs=False, ranges=None):
    """linear_regression_dims.go:23-106 — data = [x_0..x_{d-1}, y] columns.

    Output order: [N, sum x_j (d), sum x_j x_k j<=k (row-major upper tri), sum y, sum x_j y (d)]."""
    return _encrypt_with_proofs(pk, _moments("lin_reg", data, pk.device, len(data)), with_proofs, ranges)


# ----------------------------------------------------------------------------- many DPs at once
# Operations whose per-DP outputs are sums of products of record columns: the
# K14 kernel computes them for every DP of a rank in one launch.
MOMENT_OPS = ("sum", "mean", "variance", "cosim", "lin_reg", "MLeval")
# Operations encoded as 0/1 bit vectors (OR/AND encodings, OR_AND.go).
BIT_OPS = ("bool_AND", "bool_OR", "min", "max", "union", "inter")
BATCH_OPS = MOMENT_OPS + BIT_OPS + ("frequencyCount",)


def moment_pairs(name: str, C: int) -> list:
    """Column pairs (a, b) of the K14 reduction whose sums are the outputs of
    ``name``, in the reference's output order; index C is the constant 1
    (N = (C, C), sum x_a = (a, C))."""
    if name == "sum":
        return [(0, C)]
    if name == "mean":
        return [(0, C), (C, C)]
    if name == "variance":
        return [(0, C), (C, C), (0, 0)]
    if name == "cosim":
        return [(0, C), (1, C), (0, 0), (1, 1), (0, 1)]
    if name == "MLeval":  # Z = [y, pred - y]
        return [(C, C), (0, C), (0, 0), (1, 1)]
    if name == "lin_reg":  # Z = [x_0 .. x_{d-1}, y]
        d = C - 1
        return ([(C, C)] + [(j, C) for j in range(d)] + [(j, k) for j in range(d) for k in range(j, d)]
                + [(d, C)] + [(j, d) for j in range(d)])
    raise ValueError(f"{name} is not a moment operation")


def batch_values(name: str, Z: torch.Tensor, seg_rows, qmin: int = 0, qmax: int = 0) -> torch.Tensor:
    """[n_dp, n_out] int64 outputs of every DP of a batch, on Z's device.

    Z [rows, n_in] holds the DPs' records back to back (``seg_rows[g]`` rows for
    DP g, columns = the operation's input columns).  Moments: one K14 launch;
    frequency counts: one bincount over (DP, bin); bit encodings: the 0/1
    value each DP encrypts (OR-encoded bit, or the inverted AND bit), as in
    ``encode_bits`` with proofs."""
    from .. import native as nt

    G = len(seg_rows)
    dev = Z.device
    if name in MOMENT_OPS:
        if name == "MLeval":
            Z = torch.stack([Z[:, 0], Z[:, 1] - Z[:, 0]], dim=1)
        elif name in ("sum", "mean", "variance"):
            Z = Z[:, :1]
        return nt.int_moments(Z.contiguous(), seg_rows, moment_pairs(name, Z.shape[1]))
    counts = torch.as_tensor(list(seg_rows), dtype=torch.int64)
    x = Z[:, 0]
    if name in ("bool_AND", "bool_OR"):  # the DP's bit is its first record == 1 (encode_decode.go:82-118)
        first = torch.zeros(G, dtype=torch.int64, device=dev)
        if x.numel():
            starts = (counts.cumsum(0) - counts).clamp(max=x.numel() - 1).to(dev)
            first = ((x[starts] == 1) & (counts > 0).to(dev)).to(torch.int64)
        return (first if name == "bool_OR" else 1 - first)[:, None]
    seg = torch.repeat_interleave(torch.arange(G, device=dev), counts.to(dev), output_size=Z.shape[0])
    n = qmax - qmin + 1
    if name == "frequencyCount":
        keep = (x >= qmin) & (x <= qmax)
        flat = (seg * n + (x - qmin))[keep]
        return torch.bincount(flat, minlength=G * n)[: G * n].reshape(G, n)
    grid = torch.arange(qmin, qmax + 1, device=dev)
    if name in ("min", "max"):
        big = torch.iinfo(torch.int64)
        init = torch.full((G,), big.max if name == "min" else big.min, dtype=torch.int64, device=dev)
        ext = init.scatter_reduce(0, seg, x, "amin" if name == "min" else "amax", include_self=True)
        if name == "min":  # OR of bit_i = [i >= localMin]
            return (grid[None, :] >= ext[:, None]).to(torch.int64)
        return (grid[None, :] < ext[:, None]).to(torch.int64)  # inverted AND of [i >= localMax]
    if name in ("union", "inter"):
        keep = (x >= qmin) & (x <= qmax)
        hit = torch.zeros(G * n, dtype=torch.int64, device=dev)
        hit[(seg * n + (x - qmin))[keep]] = 1
        hit = hit.reshape(G, n)
        return hit if name == "union" else 1 - hit
    raise ValueError(f"{name} has no batched encoder")


def encrypt_batch(pk: eg.PublicKeyTable, values: torch.Tensor, bits: bool):
    """One encryption launch for a whole batch: ints (EncryptIntVectorGetRs),
    or for bit encodings without proofs a fresh random non-zero scalar where the
    bit absorbs and 0 elsewhere (EncryptScalar, OR_AND.go)."""
    m = values.reshape(-1).contiguous()
    if not bits:
        return eg.encrypt_ints(pk, m)
    rnd = bn.random_scalars(m.numel(), pk.device)
    s = torch.where((m != 0)[:, None], rnd, torch.zeros_like(rnd))
    return eg.encrypt_scalars(pk, s.contiguous())


# ----------------------------------------------------------------------------- boolean encodings
def encode_bits(bits, pk, mode: str, with_proofs=False, ranges=None, sig_cols=None):
    """OR_AND.go: OR-encode (mode 'or') or AND-encode ('and') a vector of bools.

    Without proofs: encrypt a random non-zero scalar for an 'absorbing' bit and
    zero otherwise (EncryptScalar); with proofs: encrypt 0/1 ints (AND
    inverted) so a [0,1] range proof applies (OR_AND.go:23-121)."""
    bits = [bool(b) for b in bits]
    if with_proofs:
        vals = [int(b) if mode == "or" else int(not b) for b in bits]
        return _encrypt_with_proofs(pk, vals, True, ranges, sig_cols)
    absorbing = [b if mode == "or" else (not b) for b in bits]
    rnd = bn.random_scalars(len(bits), pk.device)
    keep = torch.tensor(absorbing, dtype=torch.bool, device=pk.device)
    s = torch.where(keep[:, None], rnd, torch.zeros_like(rnd))
    cv, _ = eg.encrypt_scalars(pk, s.contiguous())
    clear = [int(b) if mode == "or" else int(not b) for b in bits]
    return EncodeResult(cv, clear, None)


def encode_min(data, qmin, qmax, pk, with_proofs=False, ranges=None):
    """min_max.go:13 — bit_i = [i >= localMin], OR-encoded."""
    x = _t(data[0], pk.device)
    lm = int(x.min().item())
    return encode_bits([i >= lm for i in range(qmin, qmax + 1)], pk, "or", with_proofs, ranges)


def encode_max(data, qmin, qmax, pk, with_proofs=False, ranges=None):
    """min_max.go:87 — bit_i = [i >= localMax], AND-encoded."""
    x = _t(data[0], pk.device)
    lm = int(x.max().item())
    return encode_bits([i >= lm for i in range(qmin, qmax + 1)], pk, "and", with_proofs, ranges)


def encode_union(data, qmin, qmax, pk, with_proofs=False, ranges=None):
    """set_union_intersection.go:19 — membership bits, OR-encoded."""
    present = set(int(v) for v in torch.unique(_t(data[0], pk.device)).cpu().tolist())
    return encode_bits([i in present for i in range(qmin, qmax + 1)], pk, "or", with_proofs, ranges)


def encode_inter(data, qmin, qmax, pk, with_proofs=False, ranges=None):
    """set_union_intersection.go:94 — membership bits, AND-encoded."""
    present = set(int(v) for v in torch.unique(_t(data[0], pk.device)).cpu().tolist())
    return encode_bits([i in present for i in range(qmin, qmax + 1)], pk, "and", with_proofs, ranges)


def encode_bool(data, pk, mode, with_proofs=False, ranges=None):
    """encode_decode.go:82-118: the DP's bit is datas[0][0] == 1."""
    x = data[0]
    first = int(x[0].item() if isinstance(x, torch.Tensor) else x[0])
    return encode_bits([first == 1], pk, mode, with_proofs, ranges)


# ----------------------------------------------------------------------------- dispatch
def encode(datas, pk: eg.PublicKeyTable, operation: Operation, ranges=None, with_proofs: bool = False,
           lr_data=None) -> EncodeResult:
    """encode_decode.go:14 Encode (+ EncodeForFloat :234 for logistic regression)."""
    name = operation.NameOp
    qmin, qmax = operation.QueryMin, operation.QueryMax
    if name == "sum":
        return encode_sum(datas, pk, with_proofs, ranges)
    if name == "mean":
        return encode_mean(datas, pk, with_proofs, ranges)
    if name == "variance":
        return encode_variance(datas, pk, with_proofs, ranges)
    if name == "cosim":
        return encode_cosim(datas, pk, with_proofs, ranges)
    if name == "lin_reg":
        return encode_lin_reg(datas, pk, with_proofs, ranges)
    if name == "frequencyCount":
        return encode_frequency_count(datas, qmin, qmax, pk, with_proofs, ranges)
    if name == "bool_AND":
        return encode_bool(datas, pk, "and", with_proofs, ranges)
    if name == "bool_OR":
        return encode_bool(datas, pk, "or", with_proofs, ranges)
    if name == "min":
        return encode_min(datas, qmin, qmax, pk, with_proofs, ranges)
    if name == "max":
        return encode_max(datas, qmin, qmax, pk, with_proofs, ranges)
    if name == "union":
        return encode_union(datas, qmin, qmax, pk, with_proofs, ranges)
    if name == "inter":
        return encode_inter(datas, qmin, qmax, pk, with_proofs, ranges)
    if name == "MLeval":
        return encode_model_evaluation(datas, pk, with_proofs, ranges)
    if name == "logistic regression":
        from ..models.logistic_regression import encode_logistic_regression

        X, y = lr_data
        return encode_logistic_regression(X, y, operation.LRParameters, pk, with_proofs, ranges)
    raise ValueError(f"unknown operation {name}")


# ----------------------------------------------------------------------------- decoders
def _dec(values):
    return [int(v) for v in values]


def decode_values(name: str, vals: list, operation: Operation) -> list:
    """Decoders that only need the decrypted integers (encode_decode.go:163-231)."""
    if name == "sum":
        return [float(vals[0])]
    if name == "mean":
        return [vals[0] / vals[1]]
    if name == "variance":
        mean = vals[0] / vals[1]
        return [vals[2] / vals[1] - mean * mean]
    if name == "cosim":
        sa, sb, saa, sbb, sab = vals
        return [sab / ((saa ** 0.5) * (sbb ** 0.5))]
    if name == "frequencyCount":
        return [float(v) for v in vals]
    if name == "lin_reg":
        return decode_lin_reg(vals)
    if name == "MLeval":
        return [decode_model_evaluation(vals)]
    return [float(v) for v in vals]


def decode_model_evaluation(vals) -> float:
    """model_evaluation.go:81: 1 - SSE / (sum y^2 - (sum y)^2 / N) with Go int division."""
    n, sy, syy, sse = vals
    if n == 0:
        return 0.0
    t = sy * sy
    q = t // n if (t >= 0) == (n > 0) else -((-t) // n)  # Go int64 division truncates toward zero
    denom = float(syy) - float(q)
    return 1.0 - sse / denom if denom else 0.0


def decode_lin_reg(vals) -> list:
    """linear_regression_dims.go:110-162: exact rational Gaussian elimination."""
    L = len(vals)
    # (d^2 + 5d + 4)/2 = L  ->  d
    d = int(round((-5 + (25 - 4 * (4 - 2 * L)) ** 0.5) / 2))
    A = [[Fraction(0)] * (d + 2) for _ in range(d + 1)]
    idx = 0
    for i in range(d + 1):
        for j in range(i, d + 1):
            A[i][j] = Fraction(vals[idx])
            A[j][i] = Fraction(vals[idx])
            idx += 1
    for i in range(d + 1):
        A[i][d + 1] = Fraction(vals[idx])
        idx += 1
    n = d + 1
    for c in range(n):
        piv = next((r for r in range(c, n) if A[r][c] != 0), None)
        if piv is None:
            continue
        A[c], A[piv] = A[piv], A[c]
        for r in range(n):
            if r != c and A[r][c] != 0:
                f = A[r][c] / A[c][c]
                A[r] = [a - f * b for a, b in zip(A[r], A[c])]
    return [float(A[i][n] / A[i][i]) if A[i][i] != 0 else 0.0 for i in range(n)]


def decode(cv: eg.CipherVector, secret: int, operation: Operation, table: Optional[eg.DecryptionTable] = None):
    """encode_decode.go:163 Decode."""
    name = operation.NameOp
    if name in ("bool_AND", "bool_OR", "min", "max", "union", "inter"):
        nz = eg.decrypt_check_zero(secret, cv).cpu().tolist()
        if name == "bool_OR":
            return [float(nz[0] != 0)]
        if name == "bool_AND":
            return [float(nz[0] == 0)]
        if name == "min":  # first OR-set bit
            return [float(next((i for i, b in enumerate(nz) if b != 0), 0) + operation.QueryMin)]
        if name == "max":  # first AND-true bit
            return [float(next((i for i, b in enumerate(nz) if b == 0), 0) + operation.QueryMin)]
        if name == "union":
            return [float(b != 0) for b in nz]
        return [float(b == 0) for b in nz]
    table = table or eg.decryption_table(10000, cv.device)
    vals = _dec(eg.decrypt_auto(secret, cv, table.bound).cpu().tolist())
    if name == "logistic regression":
        from ..models.logistic_regression import decode_logistic_regression_values

        return decode_logistic_regression_values(vals, operation.LRParameters)
    return decode_values(name, vals, operation)
