"""Logging, environment and rank helpers (reference: /root/reference/src/utils.py)."""
from .log import Level, print_d, set_verbosity, get_verbosity  # noqa: F401
from .env import eval_arg, DistEnv, dist_env_from_environ  # noqa: F401
