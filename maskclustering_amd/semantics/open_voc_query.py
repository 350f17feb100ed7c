"""Drop-in for the reference's ``semantics/open-voc_query.py``.

``main(args)`` keeps the reference's inputs and output file (open-voc_query.py:8-57): the
exported ``object_dict.npy``, the per-mask CLIP features ``open-vocabulary_features.npy``, the
dataset's label text features and label ids, written to
``data/prediction/<config>/<seq_name>.npz`` as ``pred_masks`` / ``pred_score`` / ``pred_classes``.
``query(...)`` is its compute: every object's label on the device in one C-ABI call
(``mc_openvoc_query``, include/mcgraph.h): the mean of the representative masks' features, the
similarities with all label features, exp(100 sim), the softmax and the first argmax
(:32-50), one workgroup per object.  The similarity dot products are summed in float64 and
rounded once (numpy's float32 BLAS order is its own), so a label can differ from numpy's only
where two labels' probabilities are within a few float32 ULP (tests/test_gpu_openvoc.py).

Objects with no representative mask keep class 0 and an empty mask column (:33-34), as in the
reference.  A feature missing from ``open-vocabulary_features.npy`` raises KeyError (:37).
"""
from __future__ import annotations

import os

import numpy as np

from maskclustering_amd import _device  # absolute: also run as `semantics.open-voc_query`

TEMPERATURE = 100.0  # exp_sim = np.exp(raw_similarity * 100) (:42)


def query(object_dict, clip_feature, label_features_dict, label2id, total_point_num):
    """open-voc_query.py:13-51 without the file IO: returns the reference's pred_dict."""
    label_text_features = np.stack(list(label_features_dict.values()))           # :13
    descriptions = list(label_features_dict.keys())
    num_instance = len(object_dict)
    pred = {"pred_masks": np.zeros((total_point_num, num_instance), dtype=bool),  # :24-28
            "pred_score": np.ones(num_instance),
            "pred_classes": np.zeros(num_instance, dtype=np.int32)}
    rows, row_of, off = [], {}, [0]
    obj_rows = []
    for value in object_dict.values():
        for mask_info in value["repre_mask_list"]:
            key = f"{mask_info[0]}_{mask_info[1]}"
            r = row_of.get(key)
            if r is None:
                r = row_of[key] = len(rows)
                rows.append(clip_feature[key])                                   # KeyError as at :37
            obj_rows.append(r)
        off.append(len(obj_rows))
    if num_instance == 0:
        return pred
    dim = label_text_features.shape[1]
    feats = np.stack(rows).astype(np.float32) if rows else np.zeros((0, dim), np.float32)
    if rows and feats.shape[1] != dim:
        raise ValueError(f"shapes {feats.shape[1:]} and {label_text_features.shape[1:]} not aligned")  # np.dot
    ctx = _device.context()
    lab = ctx.openvoc_query(np.array(off, np.int64), np.array(obj_rows, np.int32), feats,
                            label_text_features.astype(np.float32), TEMPERATURE)
    for idx, (key, value) in enumerate(object_dict.items()):
        if lab[idx] < 0:                                                          # :33-34
            continue
        pred["pred_classes"][idx] = label2id[descriptions[int(lab[idx])]]         # :47-48
        point_ids = value["point_ids"]
        pred["pred_masks"][list(point_ids), idx] = True                          # :50-53
    return pred


def main(args, dataset=None):
    """open-voc_query.py:8-57 (``dataset`` defaults to the reference's ``utils.config.get_dataset``)."""
    if dataset is None:
        from utils.config import get_dataset  # the reference checkout's dataset layer
        dataset = get_dataset(args)
    total_point_num = dataset.get_scene_points().shape[0]
    label_features_dict = dataset.get_label_features()
    base = f"{dataset.object_dict_dir}/{args.config}"
    object_dict = np.load(f"{base}/object_dict.npy", allow_pickle=True).item()
    clip_feature = np.load(f"{base}/open-vocabulary_features.npy", allow_pickle=True).item()
    label2id = dataset.get_label_id()[0]
    pred_dir = os.path.join("data/prediction", args.config)
    os.makedirs(pred_dir, exist_ok=True)
    pred = query(object_dict, clip_feature, label_features_dict, label2id, total_point_num)
    np.savez(f"{pred_dir}/{args.seq_name}.npz", **pred)


if __name__ == "__main__":  # python -m semantics.open-voc_query --config ... --seq_name ... (run.py:102)
    from utils.config import get_args
    main(get_args())
