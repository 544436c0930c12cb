from .memory import print_memory_stats  # noqa: F401
from .utils import get, set_seed  # noqa: F401
