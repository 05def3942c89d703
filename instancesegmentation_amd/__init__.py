"""MI355X-native (gfx950) train/infer path for the YanMiaoW/instanceSegmentation model.

    from instancesegmentation_amd.model.segment import Segment   # drop-in for model.segment

All arithmetic runs in libisg.so (hand-written HIP kernels, include/isg.h); the
Python layer records and replays fused op lists (engine.py, runtime.py).
"""
__version__ = "0.1.0"
