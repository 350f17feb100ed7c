"""Golden fixture for the open-vocabulary query: the REFERENCE's own
``semantics/open-voc_query.py`` ``main(args)`` run on synthetic inputs, its output npz captured.

Run ONLY in the build container, where /root/reference exists:

    python tests/golden/make_openvoc_golden.py

The reference module is loaded from its file with a stand-in ``utils.config`` (its dataset layer
reads ScanNet files and Open3D meshes; here a small object serves the five things main() reads:
get_scene_points, get_label_features, get_label_id, object_dict_dir, and the args).  The inputs
main() np.loads (object_dict.npy, open-vocabulary_features.npy) are written by this script into a
temporary directory; the reference's code is otherwise unmodified.  Stored: the inputs (features
as float16-exact values so the file stays small; the reference computes on them as float32, as
CLIP's extractor writes them) and the reference's pred_classes / pred_masks.  Data only.

Cases: objects with 0-5 representative masks, shared masks, two label text features that are
equal (an exact probability tie: np.argmax takes the first), an object whose feature equals a
label's (exp(100 sim) overflows to inf, inf / inf = NaN: np.argmax takes the first NaN), and an
object whose feature is near two labels at once.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import tempfile
import types
from types import SimpleNamespace

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
D, L, P, NOBJ = 1024, 198, 3000, 48


def _unit16(v):
    v = v / np.linalg.norm(v, axis=-1, keepdims=True)
    return v.astype(np.float16).astype(np.float32)


def make_inputs(seed=0):
    rng = np.random.default_rng(seed)
    labels = _unit16(rng.standard_normal((L, D)))
    labels[17] = labels[5]                                   # exact tie between labels 5 and 17
    descriptions = [f"label_{i:03d}" for i in range(L)]
    ids = rng.permutation(np.arange(1, 1000))[:L]
    keys, feats = [], []

    def feat(v):
        keys.append(f"{10 * len(keys)}_{1 + len(keys) % 7}")
        feats.append(v.astype(np.float32))
        return len(keys) - 1

    base = [feat(_unit16(rng.standard_normal(D) + 3.0 * labels[rng.integers(L)])) for _ in range(120)]
    inf_row = feat(labels[40].copy())                        # sim ~ 1 -> exp overflow -> NaN path
    tie_row = feat(_unit16(rng.standard_normal(D) + 4.0 * labels[5]))
    two_row = feat(_unit16(labels[60] + labels[61]))
    objects = []
    for k in range(NOBJ):
        nm = int(rng.integers(0, 6)) if k % 9 else 0
        rows = [int(r) for r in rng.choice(base, nm, replace=False)] if nm else []
        if k == 3:
            rows = [inf_row]
        if k == 4:
            rows = [tie_row, tie_row]
        if k == 5:
            rows = [two_row]
        if k == 6:
            rows = [inf_row, tie_row, base[0]]
        pts = np.unique(rng.integers(0, P, int(rng.integers(1, 200))))
        objects.append((rows, pts))
    return dict(labels=labels, descriptions=descriptions, ids=ids, keys=keys, feats=np.stack(feats),
                objects=objects)


def _object_dict(inp):
    od = {}
    for k, (rows, pts) in enumerate(inp["objects"]):
        ml = [(int(inp["keys"][r].split("_")[0]), int(inp["keys"][r].split("_")[1]), 0.5) for r in rows]
        od[k] = {"point_ids": [int(p) for p in pts], "mask_list": ml, "repre_mask_list": ml}
    return od


def main():
    inp = make_inputs()
    od = _object_dict(inp)
    clip = {k: f for k, f in zip(inp["keys"], inp["feats"])}
    lab = {d: inp["labels"][i] for i, d in enumerate(inp["descriptions"])}
    label2id = {d: int(i) for d, i in zip(inp["descriptions"], inp["ids"])}
    with tempfile.TemporaryDirectory() as tmp:
        obj_dir = os.path.join(tmp, "objects")
        os.makedirs(os.path.join(obj_dir, "cfg"))
        np.save(os.path.join(obj_dir, "cfg", "object_dict.npy"), od, allow_pickle=True)
        np.save(os.path.join(obj_dir, "cfg", "open-vocabulary_features.npy"), clip, allow_pickle=True)
        ds = SimpleNamespace(get_scene_points=lambda: np.zeros((P, 3)), get_label_features=lambda: lab,
                             get_label_id=lambda: (label2id, None), object_dict_dir=obj_dir)
        utils = types.ModuleType("utils")
        cfg = types.ModuleType("utils.config")
        cfg.get_dataset = lambda args: ds
        cfg.get_args = lambda: None
        utils.config = cfg
        sys.modules["utils"], sys.modules["utils.config"] = utils, cfg
        sys.dont_write_bytecode = True
        spec = importlib.util.spec_from_file_location("ref_open_voc_query",
                                                      os.path.join(REF, "semantics", "open-voc_query.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        cwd = os.getcwd()
        os.chdir(tmp)
        try:
            mod.main(SimpleNamespace(config="cfg", seq_name="scene"))
        finally:
            os.chdir(cwd)
        got = dict(np.load(os.path.join(tmp, "data", "prediction", "cfg", "scene.npz")))
    obj_off = np.zeros(NOBJ + 1, np.int64)
    np.cumsum([len(r) for r, _ in inp["objects"]], out=obj_off[1:])
    pt_off = np.zeros(NOBJ + 1, np.int64)
    np.cumsum([len(p) for _, p in inp["objects"]], out=pt_off[1:])
    out = dict(labels=inp["labels"].astype(np.float16), descriptions=np.array(inp["descriptions"]),
               label_ids=inp["ids"].astype(np.int32), keys=np.array(inp["keys"]),
               feats=inp["feats"].astype(np.float16), obj_off=obj_off,
               obj_rows=np.concatenate([np.array(r, np.int32) for r, _ in inp["objects"]]),
               pt_off=pt_off, pt_idx=np.concatenate([p for _, p in inp["objects"]]).astype(np.int32),
               num_points=np.array(P), pred_classes=got["pred_classes"],
               pred_masks_packed=np.packbits(got["pred_masks"], axis=0), pred_score=got["pred_score"])
    path = os.path.join(HERE, "openvoc_small.npz")
    np.savez_compressed(path, **out)
    print(f"objects={NOBJ} classes={got['pred_classes'].tolist()} -> {path} {os.path.getsize(path) / 1e3:.1f} kB")


if __name__ == "__main__":
    main()
