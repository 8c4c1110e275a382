"""Remote-execution surface the aggregation method sits behind (mirror of substrafl/remote/).

Only what the hot path's callers need: the ``@remote`` / ``@remote_data`` decorators
(decorators.py:18-143), ``RemoteOperation`` (operations.py:13-27), ``RemoteStruct``
(remote_struct.py:12-137), the task-process adapter ``RemoteMethod`` (substratools_methods.py:18-166)
and the pickle wire format (serializers/pickle_serializer.py:8-33).
"""

from .decorators import remote, remote_data  # noqa: F401
from .operations import RemoteDataOperation, RemoteOperation  # noqa: F401
from .remote_struct import RemoteStruct  # noqa: F401
from .serializers import PickleSerializer  # noqa: F401
from .substratools_methods import InputIdentifiers, OutputIdentifiers, RemoteMethod  # noqa: F401
