"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

This package restates, in plain numpy / C, the reference algorithms of the
non-rigid TSDF fusion hot path of remmel/OcclusionFusion:

  * TSDFVolume geometry + CPU integrate      (fusion_with_occlusion/tsdf.py)
  * WarpField.skin (k-NN skinning)           (fusion_with_occlusion/warpfield.py)
  * ED_warp / Registration.deform_ED         (NonRigidICP/model/geometry.py, registration_fusion.py)
  * DeformNet.optimize Gauss-Newton          (model/model.py)

It is the CHECKER for the HIP product path. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
or execute anything in here; the product package ``occlusionfusion_amd`` never
does, and fails loudly when its HIP library is missing.

Pinning status:
  * skinning k-NN  — pinned against the reference's own compiled C++
    ``compute_pixel_anchors_euclidean`` (csrc/cpu/graph_proc.cpp:610-709),
    built from /root/reference sources into ``oracle/_ref`` by
    ``oracle/build_ref.py``; golden vectors in ``tests/golden``.
  * integrate / warp / GN — the reference Python cannot be imported here
    (numba, open3d, pykdtree, skimage, kornia, lietorch are absent: ordinary
    ImportErrors) and the reference holds no asserting tests, so these are
    restatements pinned only by closed-form known-answer tests:
    **parity unpinned** against reference outputs.
"""
