from .secret_sharing import AdditiveSecretSharing, SecretSharing, ss_params

__all__ = ['AdditiveSecretSharing', 'SecretSharing', 'ss_params']
