from .dataset import VideoCaptionDataset, CaptionLoader
from .synthetic import make_synthetic, make_splits, MSRVTT_FEAT_DIMS, MSVD_FEAT_DIMS
from . import formats

__all__ = ['VideoCaptionDataset', 'CaptionLoader', 'make_synthetic', 'make_splits',
           'MSRVTT_FEAT_DIMS', 'MSVD_FEAT_DIMS', 'formats']
