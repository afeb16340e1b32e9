"""Spatial transformer (reference nn/network/stn.py:5-23).

In this build the translation-only STN used by PhysicsNet's decoder is fused
with compositing and the loss into ``paig_decoder_fwd/bwd``
(csrc/decoder.hip), which reproduces affine_grid's fp64 grid (Q9) and
grid_sample's bilinear / zeros / align_corners=False sampling.  The general
affine ``stn`` / ``batch_transformer`` helpers are never called on the
reference's path and are not provided."""
