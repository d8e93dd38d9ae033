"""Build the reference's own C++ ``csrc`` (NeuralNRT._C) into ``oracle/_ref`` — TEST INFRASTRUCTURE ONLY.

Compiles, from the sources where they lie under /root/reference (never copied):
  csrc/main.cpp, csrc/cpu/graph_proc.cpp, csrc/cpu/image_proc.cpp
with the vendored Eigen at NonRigidICP/external. The resulting
extension module is used only to pin the oracle's skinning k-NN
(``compute_pixel_anchors_euclidean``, graph_proc.cpp:610-709) and to generate
graph fixtures (``sample_nodes``, ``compute_edges_euclidean``).

Outputs go only to oracle/_ref/ (git-ignored). Usage: python -m oracle.build_ref
"""
import os
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "_ref")
NAME = "NeuralNRT_C_ref"


def build(verbose=False):
    if not os.path.isdir(os.path.join(REF, "csrc")):
        raise FileNotFoundError("reference sources not present (expected on the CPU build container only)")
    import torch  # noqa: F401  (torch must be imported before the extension)
    from torch.utils.cpp_extension import load
    os.makedirs(OUT, exist_ok=True)
    return load(name=NAME,
                sources=[os.path.join(REF, "csrc/main.cpp"),
                         os.path.join(REF, "csrc/cpu/graph_proc.cpp"),
                         os.path.join(REF, "csrc/cpu/image_proc.cpp")],
                extra_include_paths=[os.path.join(REF, "csrc"), os.path.join(REF, "NonRigidICP/external")],
                extra_cflags=["-O3", "-std=c++17", "-fopenmp"], extra_ldflags=["-fopenmp"],
                build_directory=OUT, verbose=verbose)


def load_prebuilt():
    """Import the already built module from oracle/_ref (works without /root/reference)."""
    import importlib.util
    import torch  # noqa: F401
    path = os.path.join(OUT, NAME + ".so")
    if not os.path.exists(path):
        return None
    spec = importlib.util.spec_from_file_location(NAME, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


if __name__ == "__main__":
    m = build(verbose="-v" in sys.argv)
    print("built", m.__file__)
