"""(De)serialisation of parity fixtures in tests/golden/*.npz (plain arrays,
loaded with allow_pickle=False)."""
import numpy as np

from dm._ffi import DmParams

PARAM_FIELDS = [name for name, _ in DmParams._fields_]


def dump_case(arrays, name, params, batches, amin, inc, counts, L, state, mask, labels, clusters):
    for f in PARAM_FIELDS:
        arrays[f"{name}__p_{f}"] = np.array(getattr(params, f))
    arrays[f"{name}__nbatch"] = np.array(len(batches))
    for k, (poses, ranges) in enumerate(batches):
        arrays[f"{name}__poses{k}"] = np.asarray(poses, np.float64)
        arrays[f"{name}__ranges{k}"] = np.asarray(ranges, np.float32)
    arrays[f"{name}__amin"] = np.array(amin, np.float32)
    arrays[f"{name}__inc"] = np.array(inc, np.float32)
    arrays[f"{name}__counts"] = np.asarray(counts, np.int64)
    arrays[f"{name}__L"] = L
    arrays[f"{name}__state"] = state
    arrays[f"{name}__mask"] = mask
    arrays[f"{name}__labels"] = labels
    arrays[f"{name}__clusters"] = clusters


def load_case(d, name):
    p = DmParams()
    for f in PARAM_FIELDS:
        setattr(p, f, d[f"{name}__p_{f}"].item())
    nb = int(d[f"{name}__nbatch"])
    return {
        "params": p,
        "batches": [(d[f"{name}__poses{k}"], d[f"{name}__ranges{k}"]) for k in range(nb)],
        "amin": float(d[f"{name}__amin"]),
        "inc": float(d[f"{name}__inc"]),
        "counts": d[f"{name}__counts"],
        "L": d[f"{name}__L"],
        "state": d[f"{name}__state"],
        "mask": d[f"{name}__mask"],
        "labels": d[f"{name}__labels"],
        "clusters": d[f"{name}__clusters"],
    }
