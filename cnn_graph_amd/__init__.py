"""cnn_graph_amd -- MI355X-native Chebyshev spectral graph convolution.

A drop-in for the hot path of xu-wang11/cnn_graph: ``GraphConv.chebyshev5`` /
``cgcnn.chebyshev5`` / ``filter.cheby_conv`` (lib/graph_conv.py:144-176), with
the K-step recurrence, the weight contraction and the backward as hand-written
HIP kernels for gfx950 behind a C ABI (include/cheb_mi355.h), plus the graph
pooling / permutation ops around it and data-parallel gradient exchange.

Modules
  graph       host Laplacian math (lib/graph.py API)
  plan        device plan of L~ (the TF graph constant of lib/graph_conv.py:148-153)
  ops         torch autograd ops over the HIP kernels
  graph_conv  GraphConv filter plumbing (name-bound chebyshev5, residual stack)
  filter      functional cheby_conv (lib/filter.py API)
  coarsening  graph coarsening + perm_data (lib/coarsening.py API)
  dist        one-process-per-GPU data parallelism (RCCL all-reduce)
"""
__version__ = "0.1.0"

__all__ = ["graph", "plan", "ops", "graph_conv", "filter", "coarsening", "dist"]
