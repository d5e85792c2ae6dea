from .config import MODELS, EncoderConfig, get_config  # noqa: F401
