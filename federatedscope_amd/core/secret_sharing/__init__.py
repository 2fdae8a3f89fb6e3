from .secret_sharing import ss_params

__all__ = ['ss_params']
