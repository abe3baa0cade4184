"""Dataset cleaning for the logistic-regression benchmarks.

Reference: data/clean_data.py:17-91 ``cleanData(dataset, filename, label_type)``:
label in column 0; PCS drops its index column and the two trailing unused
columns; GAS_SENSOR_MULTI strips ``index:`` prefixes; MNIST rescales pixels to
[0.001, 1.0]; rows with a non-numeric feature are dropped.  The cleaned file is
``label,f1,...,fd`` per line (what ``load_csv_dataset`` reads).
"""
from __future__ import annotations

import sys

DATASETS = ("PIMA", "PCS", "SPECTF", "MNIST", "GAS_SENSOR_MULTI", "GAS_SENSOR")


def clean_rows(dataset: str, lines: list, label_type=int):
    """-> (X rows of floats, y labels, number of dropped lines)."""
    dataset = dataset.upper()
    if dataset not in DATASETS:
        raise ValueError(f"unknown dataset: {dataset}")
    rows = [ln.split(",") for ln in lines if ln != ""]
    if dataset == "PCS":
        for r in rows:
            for idx in (11, 10, 0):
                if idx < len(r):
                    del r[idx]
    elif dataset == "GAS_SENSOR_MULTI":
        rows = [[v if i == 0 else v.split(":")[1] for i, v in enumerate(r)] for r in rows]
    X, y, dropped = [], [], 0
    for r in rows:
        try:
            lab = label_type(r[0])
            feats = [float(v) for v in r[1:]]
        except ValueError:
            dropped += 1
            continue
        X.append(feats)
        y.append(lab)
    if dataset == "MNIST":
        X = [[v / 255.0 * 0.999 + 0.001 for v in r] for r in X]
    return X, y, dropped


def clean_file(dataset: str, src: str, dst: str | None = None, label_type: str = "int") -> int:
    """cleanData: rewrite ``src`` (or write ``dst``) in clean form; returns the dropped-line count."""
    lt = {"int": int, "float": float}.get(label_type)
    if lt is None:
        raise ValueError(f"unknown label type {label_type}")
    with open(src) as f:
        lines = f.read().split("\n")
    X, y, dropped = clean_rows(dataset, lines, lt)
    if dropped:
        print(f"/!\\ {dropped} line(s) dropped in {src}", file=sys.stderr)
    with open(dst or src, "w") as f:
        for feats, lab in zip(X, y):
            f.write(str(lab) + "," + ",".join(str(v) for v in feats) + "\n")
    return dropped


if __name__ == "__main__":  # python -m drynx_amd.models.datasets PCS file.txt [int|float] [out]
    a = sys.argv[1:]
    clean_file(a[0], a[1], a[3] if len(a) > 3 else None, a[2] if len(a) > 2 else "int")


def load_dp_file(path: str, op, device="cpu"):
    """A data provider's records for ``op`` from a file (the file loader of
    ``server data-provider new file-loader PATH``): one record per line,
    values separated by commas.  Logistic regression reads the cleaned
    dataset layout ``label,f1,...,fd`` (``load_csv_dataset``, the reference's
    GetDataForDataProvider) -> (X float64 [n, d], y int64 [n]); every other
    operation takes the first NbrInput values of each record as int64
    columns -> [column tensors] (the layout of ``generate_fake_data``)."""
    import numpy as np
    import torch

    if op.NameOp == "logistic regression":
        from .logistic_regression import load_csv_dataset

        X, y = load_csv_dataset(path)
        d = int(op.LRParameters.NbrFeatures)
        if X.shape[1] != d:
            raise ValueError(f"{path}: {X.shape[1]} features per record, the query has {d}")
        return X.to(device), y.to(device)
    data = np.loadtxt(path, delimiter=",", dtype=np.float64, ndmin=2)
    n_in = max(1, int(op.NbrInput))
    if data.shape[1] < n_in:
        raise ValueError(f"{path}: {data.shape[1]} values per record, the operation reads {n_in}")
    if not np.all(data[:, :n_in] == np.round(data[:, :n_in])):
        raise ValueError(f"{path}: the operation {op.NameOp} reads integer values")
    t = torch.tensor(data[:, :n_in].T.copy(), dtype=torch.int64, device=device)
    return list(t.unbind(0))
