"""Epoch logger writing the reference's ``progress.txt`` TSV (rf/src/native/python/utils/logger.py:103-448).

Same file layout so the reference's plotting / TensorBoard tools keep working:
header row of column names, one tab-separated row per epoch, ``config.json`` from
``save_config``.  Extra columns (throughput, phase timings) are appended by the
runtime.
"""
from __future__ import annotations

import atexit
import json
import os
import os.path as osp
import time
from typing import Any, Dict, List, Optional

import numpy as np


def convert_json(obj):
    """Best-effort JSON-serialisable view of arbitrary objects (for save_config)."""
    if isinstance(obj, (bool, int, float, str)) or obj is None:
        return obj
    if isinstance(obj, dict):
        return {str(k): convert_json(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [convert_json(x) for x in obj]
    if isinstance(obj, np.ndarray):
        return obj.tolist() if obj.size < 64 else f"ndarray{obj.shape}"
    if hasattr(obj, "__name__") and not hasattr(obj, "__dict__"):
        return convert_json(obj.__name__)
    if hasattr(obj, "__dict__") and obj.__dict__:
        return {str(obj): {k: convert_json(v) for k, v in obj.__dict__.items() if not k.startswith("_")}}
    return str(obj)


def statistics_scalar(x, with_min_and_max: bool = False):
    """Mean / population std (/ min / max) of a flat array (BaseReplayBuffer.py:30-53)."""
    x = np.asarray(x, dtype=np.float64).ravel()
    n = max(len(x), 1)
    mean = x.sum() / n
    std = np.sqrt(((x - mean) ** 2).sum() / n)
    if with_min_and_max:
        mn = x.min() if len(x) else np.inf
        mx = x.max() if len(x) else -np.inf
        return mean, std, mn, mx
    return mean, std


class Logger:
    def __init__(self, output_dir: Optional[str] = None, output_fname: str = "progress.txt",
                 exp_name: Optional[str] = None, quiet: bool = False):
        self.output_dir = output_dir or f"/tmp/experiments/{int(time.time())}"
        os.makedirs(self.output_dir, exist_ok=True)
        self.output_file = open(osp.join(self.output_dir, output_fname), "w")
        atexit.register(self.close)
        self.first_row = True
        self.log_headers: List[str] = []
        self.log_current_row: Dict[str, Any] = {}
        self.exp_name = exp_name
        self.quiet = quiet

    def close(self):
        if self.output_file is not None and not self.output_file.closed:
            self.output_file.close()

    def log(self, msg: str):
        if not self.quiet:
            print(msg, flush=True)

    def log_tabular(self, key: str, val):
        if self.first_row:
            self.log_headers.append(key)
        elif key not in self.log_headers:
            raise KeyError(f"new key {key!r} introduced after the first row")
        if key in self.log_current_row:
            raise KeyError(f"{key!r} already set this epoch (missing dump_tabular?)")
        self.log_current_row[key] = val

    def save_config(self, config: Dict[str, Any]):
        cj = convert_json(config)
        if self.exp_name is not None:
            cj["exp_name"] = self.exp_name
        text = json.dumps(cj, separators=(",", ":\t"), indent=4, sort_keys=True)
        with open(osp.join(self.output_dir, "config.json"), "w") as f:
            f.write(text)

    def dump_tabular(self) -> Dict[str, Any]:
        vals = [self.log_current_row.get(k, "") for k in self.log_headers]
        if not self.quiet:
            w = max(15, max(len(k) for k in self.log_headers))
            line = "-" * (22 + w)
            rows = [line]
            for k, v in zip(self.log_headers, vals):
                vs = f"{v:8.3g}" if hasattr(v, "__float__") else str(v)
                rows.append(f"| {k:>{w}s} | {vs:>15s} |")
            rows.append(line)
            print("\n".join(rows), flush=True)
        if self.output_file is not None and not self.output_file.closed:
            if self.first_row:
                self.output_file.write("\t".join(self.log_headers) + "\n")
            self.output_file.write("\t".join(map(str, vals)) + "\n")
            self.output_file.flush()
        row = dict(self.log_current_row)
        self.log_current_row.clear()
        self.first_row = False
        return row


class EpochLogger(Logger):
    """Accumulates per-epoch values with ``store`` and reduces them in ``log_tabular``."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.epoch_dict: Dict[str, List[Any]] = {}

    def store(self, **kwargs):
        for k, v in kwargs.items():
            self.epoch_dict.setdefault(k, []).append(v)

    def log_tabular(self, key: str, val=None, with_min_and_max: bool = False, average_only: bool = False):
        if val is not None:
            super().log_tabular(key, val)
            return
        v = self.epoch_dict.get(key, [])
        flat = np.concatenate([np.ravel(np.asarray(x, dtype=np.float64)) for x in v]) if v else np.zeros(0)
        if len(flat) == 0:
            stats = (float("nan"),) * (4 if with_min_and_max else 2)
        else:
            stats = statistics_scalar(flat, with_min_and_max)
        super().log_tabular(key if average_only else "Average" + key, float(stats[0]))
        if not average_only:
            super().log_tabular("Std" + key, float(stats[1]))
        if with_min_and_max:
            super().log_tabular("Max" + key, float(stats[3]))
            super().log_tabular("Min" + key, float(stats[2]))
        self.epoch_dict[key] = []

    def get_stats(self, key: str):
        v = self.epoch_dict.get(key, [])
        flat = np.concatenate([np.ravel(np.asarray(x, dtype=np.float64)) for x in v]) if v else np.zeros(0)
        return statistics_scalar(flat)


def setup_logger_kwargs(exp_name: str, seed: Optional[int] = None, data_dir: Optional[str] = None,
                        datestamp: bool = False) -> Dict[str, str]:
    """output_dir = data_dir/exp_name/exp_name_s{seed} (logger.py:388-448)."""
    ymd = time.strftime("%Y-%m-%d_") if datestamp else ""
    relpath = ymd + exp_name
    if seed is not None:
        sub = (time.strftime("%Y-%m-%d_%H-%M-%S") + "-" + exp_name + f"_s{seed}") if datestamp else f"{exp_name}_s{seed}"
        relpath = osp.join(relpath, sub)
    data_dir = data_dir or osp.join(os.getcwd(), "logs")
    return dict(output_dir=osp.join(data_dir, relpath), exp_name=exp_name)


def read_progress(path: str) -> Dict[str, List[float]]:
    """Parse a progress.txt back into columns (used by plot / TB tools and tests)."""
    with open(path) as f:
        header = f.readline().rstrip("\n").split("\t")
        cols = {h: [] for h in header}
        for line in f:
            parts = line.rstrip("\n").split("\t")
            for h, p in zip(header, parts):
                try:
                    cols[h].append(float(p))
                except ValueError:
                    cols[h].append(float("nan"))
    return cols
