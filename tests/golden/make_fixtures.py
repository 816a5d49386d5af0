"""Extract golden fixtures from the reference's run artifacts (run ONCE in the
build container, where /root/reference exists; the outputs are committed).

Nothing is unpickled and no reference code is imported or executed:
  * ``outputs/*/final_poses.pt`` is a zip; its ``data.pkl`` is scanned as BYTES
    for the key -> storage-id mapping (``initial_poses`` -> '0', ...) and the
    pose-error floats (pickle BINFLOAT opcodes), and ``data/<id>`` are raw
    little-endian float32 storages of shape (100, 4, 4);
  * ``logs/*.csv`` and ``summary.json`` are read as text / JSON.

Outputs: tests/golden/final_poses_<run>.npz and tests/golden/reference_artifacts.json
"""

from __future__ import annotations

import csv
import json
import re
import struct
import zipfile
from pathlib import Path

import numpy as np

REF = Path("/root/reference/outputs")
OUT = Path(__file__).resolve().parent


def _storage_keys(pkl: bytes) -> dict:
    """key name -> storage id, from the pickle byte stream (no unpickling)."""
    keys = {}
    for name in (b"initial_poses", b"optimized_poses", b"ground_truth_poses"):
        i = pkl.index(name)
        # first 1-char string after the key = the storage id ('0'/'1'/'2')
        m = re.search(rb"X\x01\x00\x00\x00(\d)", pkl[i:i + 200])
        keys[name.decode()] = m.group(1).decode()
    return keys


def _pose_errors(pkl: bytes) -> dict:
    out = {}
    for name in ("rotation_error_mean", "rotation_error_std", "rotation_error_max",
                 "translation_error_mean", "translation_error_std", "translation_error_max"):
        nb = name.encode()
        i = pkl.index(nb) + len(nb)
        j = pkl.index(b"G", i)  # BINFLOAT opcode, 8-byte big-endian double follows
        out[name] = struct.unpack(">d", pkl[j + 1:j + 9])[0]
    return out


def extract_final_poses() -> dict:
    meta = {}
    for f in sorted(REF.glob("*/final_poses.pt")):
        run = f.parent.name
        z = zipfile.ZipFile(f)
        prefix = z.namelist()[0].split("/")[0]
        pkl = z.read(f"{prefix}/data.pkl")
        keys = _storage_keys(pkl)
        arrays = {}
        for k, sid in keys.items():
            raw = z.read(f"{prefix}/data/{sid}")
            arrays[k] = np.frombuffer(raw, dtype="<f4").reshape(100, 4, 4).copy()
        np.savez_compressed(OUT / f"final_poses_{run}.npz", **arrays)
        meta[run] = {"storage_ids": keys, "pose_errors": _pose_errors(pkl)}
    return meta


def extract_logs() -> dict:
    out = {}
    for run_dir in sorted(REF.iterdir()):
        csvp = run_dir / "logs" / "train_metrics.csv"
        if not csvp.exists():
            continue
        with open(csvp) as fh:
            rows = [r for _, r in zip(range(3), csv.DictReader(fh))]
        summ = json.loads((run_dir / "summary.json").read_text()) if (run_dir / "summary.json").exists() else {}
        out[run_dir.name] = {
            "learning_rate_first_rows": [float(r["learning_rate"]) for r in rows],
            "params_per_net": summ.get("model_info", {}).get("model_coarse_total_params",
                                                              summ.get("model_coarse_total_params")),
            "config": summ.get("config"),
        }
    return out


def _pickle_strings(pkl: bytes) -> list:
    """Every BINUNICODE string of a pickle stream, in order (opcode 'X' + 4-byte length),
    read as bytes -- the key names of a saved dict, without unpickling."""
    out, i = [], 0
    while True:
        i = pkl.find(b"X", i)
        if i < 0 or i + 5 > len(pkl):
            return out
        n = struct.unpack("<I", pkl[i + 1:i + 5])[0]
        if 0 < n < 64 and i + 5 + n <= len(pkl):
            try:
                t = pkl[i + 5:i + 5 + n].decode("ascii")
                if t.isidentifier():
                    out.append(t)
                    i += 5 + n
                    continue
            except UnicodeDecodeError:
                pass
        i += 1


def extract_layout() -> dict:
    """The reference's output-folder contract per run kind (train.py vs train_pose_opt.py):
    top-level files, logs/ files, CSV headers, JSON key sets, image-name patterns and the
    key names inside final_poses.pt."""
    out = {}
    for run_dir in sorted(REF.iterdir()):
        kind = "pose_opt" if "poseopt" in run_dir.name else "train"
        rec = out.setdefault(kind, {"runs": [], "top_files": None, "log_files": set(), "csv_headers": {},
                                    "summary_keys": None, "experiment_config_keys": None, "config_keys": None,
                                    "image_patterns": set(), "final_poses_keys": None})
        rec["runs"].append(run_dir.name)
        top = sorted(f.name for f in run_dir.iterdir() if f.name != "results.txt")
        rec["top_files"] = top
        for f in sorted((run_dir / "logs").glob("*.csv")):
            rec["log_files"].add(f.name)
            rec["csv_headers"][f.name] = f.read_text().splitlines()[0]
        for name, key in (("summary.json", "summary_keys"), ("experiment_config.json", "experiment_config_keys"),
                          ("config.json", "config_keys")):
            rec[key] = sorted(json.loads((run_dir / name).read_text()).keys())
        for img in (run_dir / "images").glob("*.png"):
            rec["image_patterns"].add(re.sub(r"\d{7}", "{it:07d}", re.sub(r"^val_\d+", "val_{i}", img.name)))
        fp = run_dir / "final_poses.pt"
        if fp.exists():
            z = zipfile.ZipFile(fp)
            prefix = z.namelist()[0].split("/")[0]
            names = _pickle_strings(z.read(f"{prefix}/data.pkl"))
            rec["final_poses_keys"] = [k for k in ("initial_poses", "optimized_poses", "ground_truth_poses",
                                                   "pose_errors") if k in names]
    for rec in out.values():
        rec["log_files"] = sorted(rec["log_files"])
        rec["image_patterns"] = sorted(rec["image_patterns"])
    return out


def main():
    artifacts = {"final_poses": extract_final_poses(), "runs": extract_logs(), "layout": extract_layout()}
    (OUT / "reference_artifacts.json").write_text(json.dumps(artifacts, indent=1, sort_keys=True))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
