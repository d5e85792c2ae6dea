from .broker import Broker  # noqa: F401
from .client import (ConnectionClosedError, Msg, NatsClient, NatsError, NoRespondersError,  # noqa: F401
                     RequestTimeoutError, Subscription)
