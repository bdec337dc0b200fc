"""cake_amd — an MI355X-native, layer-sharded inference engine with cake's capabilities.

Layers: ``ops`` (gfx950 HIP kernels + PyTorch oracle), ``models``
(Llama-3, Stable Diffusion), ``parallel`` (topology, transports, master/worker
roles), ``api`` (OpenAI-compatible REST), ``utils`` (safetensors, synthesis,
metrics).  ``csrc/`` holds the HIP kernels and the C++ host runtime, built
in-tree by :mod:`cake_amd.build`.
"""
__version__ = "0.1.0"
