"""Minimal TOML writer + tomli reader for the CLI config streams
(reference cmd/client/config.go uses go-toml over stdin/stdout)."""
from __future__ import annotations

import tomli


def loads(s: str) -> dict:
    return tomli.loads(s) if s.strip() else {}


def _val(v):
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (int, float)):
        return repr(v)
    if isinstance(v, list):
        return "[" + ", ".join(_val(x) for x in v) + "]"
    return '"' + str(v).replace("\\", "\\\\").replace('"', '\\"') + '"'


def dumps(d: dict, prefix: str = "") -> str:
    out, tables = [], []
    for k, v in d.items():
        if isinstance(v, dict):
            tables.append((k, v))
        elif isinstance(v, list) and v and isinstance(v[0], dict):
            tables.append((k, v))
        elif v is not None:
            out.append(f"{k} = {_val(v)}")
    text = "\n".join(out) + ("\n" if out else "")
    for k, v in tables:
        name = f"{prefix}.{k}" if prefix else k
        if isinstance(v, dict):
            text += f"\n[{name}]\n" + dumps(v, name)
        else:
            for item in v:
                text += f"\n[[{name}]]\n" + dumps(item, name)
    return text
