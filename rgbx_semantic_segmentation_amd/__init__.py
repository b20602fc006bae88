"""MI355X-native CMX RGB-X segmentation training step (gfx950 HIP kernels behind a C-ABI)."""
__version__ = "0.1.0"
