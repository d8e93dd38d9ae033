"""CPU: the reference's graph / image .bin formats (utils/utils.py:205-383) byte for byte: the expected bytes
are built with struct exactly as the reference writer packs them ('I' header words, '={n}f' / '={n}i' payload)."""
import struct

import numpy as np

from occlusionfusion_amd import formats


def test_graph_and_image_formats_bytes(tmp_path):
    rng = np.random.default_rng(0)
    nodes = rng.random((5, 3)).astype(np.float32)
    edges = rng.integers(-1, 5, (5, 8)).astype(np.int32)
    w = rng.random((5, 8)).astype(np.float32)
    cl = rng.integers(0, 3, (5, 1)).astype(np.int32)
    img_f = rng.random((4, 6, 4)).astype(np.float32)
    img_i = rng.integers(-1, 9, (4, 6, 4)).astype(np.int32)
    cases = [
        (formats.save_graph_nodes, formats.load_graph_nodes, nodes,
         struct.pack("I", 5) + struct.pack("={}f".format(nodes.size), *nodes.flatten("C"))),
        (formats.save_graph_edges, formats.load_graph_edges, edges,
         struct.pack("I", 5) + struct.pack("I", 8) + struct.pack("={}i".format(edges.size), *edges.flatten("C"))),
        (formats.save_graph_edges_weights, formats.load_graph_edges_weights, w,
         struct.pack("I", 5) + struct.pack("I", 8) + struct.pack("={}f".format(w.size), *w.flatten("C"))),
        (formats.save_graph_clusters, formats.load_graph_clusters, cl,
         struct.pack("I", 5) + struct.pack("I", 1) + struct.pack("={}i".format(cl.size), *cl.flatten("C"))),
        (formats.save_float_image, formats.load_float_image, img_f,
         struct.pack("I", 4) + struct.pack("I", 6) + struct.pack("I", 4)
         + struct.pack("={}f".format(img_f.size), *img_f.flatten("C"))),
        (formats.save_int_image, formats.load_int_image, img_i,
         struct.pack("I", 4) + struct.pack("I", 6) + struct.pack("I", 4)
         + struct.pack("={}i".format(img_i.size), *img_i.flatten("C"))),
    ]
    for i, (save, load, arr, expected) in enumerate(cases):
        p = tmp_path / f"f{i}.bin"
        save(str(p), arr)
        assert p.read_bytes() == expected, save.__name__
        back = load(str(p))
        assert back.dtype == arr.dtype and np.array_equal(back, arr), load.__name__


def test_truncated_file_raises(tmp_path):
    p = tmp_path / "t.bin"
    p.write_bytes(struct.pack("I", 10) + b"\0" * 8)
    try:
        formats.load_graph_nodes(str(p))
    except ValueError:
        return
    raise AssertionError("truncated payload not detected")
