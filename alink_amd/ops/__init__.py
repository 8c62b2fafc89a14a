"""Hand-written HIP/CDNA4 kernels (``csrc/*.hip``) and their Python wrappers."""
