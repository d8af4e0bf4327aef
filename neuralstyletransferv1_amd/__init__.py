"""MI355X-native stylization engine for the TrentMahaffey/NeuralStyleTransferV1 hot path.

Drop-in surfaces: `transformer_net.TransformerNet`, `transformer_net_nst.TransformerNet`,
`model.ReCoNet` (nn.Module protocol), `utils.gram_matrix`, and the `pipeline` /
`run_videos` CLIs.  Compute runs in libnst_hip.so (hand-written HIP for gfx950).
"""
__version__ = "0.1.0"
