from .broker import Broker, NativeBroker, PyBroker  # noqa: F401
from .client import (ConnectionClosedError, Msg, NatsClient, NatsError, NoRespondersError,  # noqa: F401
                     RequestTimeoutError, Subscription)
