from .dist import DistContext, init_distributed, FlatGradBucket

__all__ = ['DistContext', 'init_distributed', 'FlatGradBucket']
