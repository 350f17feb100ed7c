"""Host-side logic of the drop-in modules (no GPU): imports under the
reference's names, the Node record, and the degenerate paths that return
before any device work."""
import numpy as np
import torch


def test_modules_expose_reference_names():
    from maskclustering_amd.graph import construction, iterative_clustering, node
    from maskclustering_amd.utils import mask_backprojection as mb
    for f in ("mask_graph_construction", "build_point_in_mask_matrix", "process_masks", "init_nodes",
              "get_observer_num_thresholds"):
        assert callable(getattr(construction, f))
    assert callable(iterative_clustering.iterative_clustering)
    assert callable(node.Node.create_node_from_list)
    for f in ("turn_mask_to_point", "frame_backprojection", "get_depth_mask", "crop_scene_points"):
        assert callable(getattr(mb, f))
    assert (mb.COVERAGE_THRESHOLD, mb.DISTANCE_THRESHOLD, mb.FEW_POINTS_THRESHOLD, mb.DEPTH_TRUNC) == (0.3, 0.01, 25, 20)


def test_node_merge_matches_reference_semantics():
    """graph/node.py:24-37: OR of rows, concatenated mask lists, union of point sets."""
    from maskclustering_amd.graph.node import Node
    a = Node([(0, 1)], torch.tensor([1., 0, 0, 1]), torch.tensor([0., 1, 0]), {1, 2}, (0, 0), None)
    b = Node.compact([(10, 3)], np.array([0, 1, 0, 1], bool), np.array([2]), 3, {2, 5}, (0, 1), None)
    m = Node.create_node_from_list([a, b], (1, 0))
    assert m.mask_list == [(0, 1), (10, 3)]
    assert m.point_ids == {1, 2, 5}
    assert m.son_node_info == {(0, 0), (0, 1)}
    assert m.visible_frame.cpu().tolist() == [1., 1., 0., 1.]
    assert m.contained_mask.cpu().tolist() == [0., 1., 1.]
    assert m.node_info == (1, 0)


def test_iterative_clustering_without_thresholds_returns_nodes():
    from maskclustering_amd.graph.iterative_clustering import iterative_clustering
    nodes = [object(), object()]
    assert iterative_clustering(nodes, [], 0.9, False) is nodes


def test_turn_mask_to_point_inf_pose_returns_early():
    """mask_backprojection.py:73-74 returns ({}, [], set()) before touching the device."""
    from maskclustering_amd.utils.mask_backprojection import turn_mask_to_point

    class DS:
        def get_intrinsics(self, f):
            return np.array([500.0, 500.0, 32.0, 24.0])

        def get_extrinsic(self, f):
            T = np.eye(4)
            T[0, 3] = np.inf
            return T

    assert turn_mask_to_point(DS(), np.zeros((5, 3)), np.zeros((48, 64), np.uint8), 0) == ({}, [], set())


def test_install_routes_reference_module_names(tmp_path):
    """With a reference-shaped tree on sys.path, install() makes main.py's imports
    (main.py:4-5) resolve to the drop-ins while other modules stay the reference's."""
    import subprocess
    import sys
    import textwrap
    from conftest import REPO
    (tmp_path / "graph").mkdir()
    (tmp_path / "utils").mkdir()
    (tmp_path / "utils" / "__init__.py").write_text("")
    (tmp_path / "utils" / "geometry.py").write_text("MARK = 'reference'\n")
    (tmp_path / "semantics").mkdir()
    code = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {str(tmp_path)!r})  # the reference checkout (cwd of main.py)
        from graph.construction import mask_graph_construction
        from graph.iterative_clustering import iterative_clustering
        from utils.mask_backprojection import frame_backprojection
        from utils.geometry import MARK
        assert mask_graph_construction.__module__ == 'maskclustering_amd.graph.construction'
        assert iterative_clustering.__module__ == 'maskclustering_amd.graph.iterative_clustering'
        assert frame_backprojection.__module__ == 'maskclustering_amd.utils.mask_backprojection'
        assert MARK == 'reference'
        import importlib.util
        spec = importlib.util.find_spec('semantics.open-voc_query')   # what `python -m` runs (run.py:102)
        assert spec.origin.endswith('maskclustering_amd/semantics/open_voc_query.py'), spec.origin
        print('ok')
    """)
    import os
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(REPO, "integration"), REPO]))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=str(tmp_path), env=env)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stderr


def test_seg_ids_above_255_raise():
    """Mask images are uint8 (mask_predict.py:102); 16-bit ids above 255 would wrap and merge masks."""
    import numpy as np
    import pytest as _pt
    from maskclustering_amd._device import seg_u8
    a = np.array([[0, 3], [255, 7]], np.uint16)
    assert seg_u8(a).dtype == np.uint8 and seg_u8(a).tolist() == [[0, 3], [255, 7]]
    with _pt.raises(ValueError):
        seg_u8(np.array([[0, 256]], np.uint16))
    with _pt.raises(ValueError):
        seg_u8(np.array([[0, 1.5]]))
