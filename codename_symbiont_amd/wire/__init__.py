from .models import *  # noqa: F401,F403
from .models import ALL_CONTRACTS, WireError, WireModel, current_timestamp_ms, generate_uuid  # noqa: F401
from . import subjects  # noqa: F401
