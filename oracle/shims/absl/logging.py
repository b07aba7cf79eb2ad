"""absl.logging -> stdlib logging (import shim for oracle/make_golden.py only)."""
import logging as _l

_log = _l.getLogger("reference")
info = _log.info
warning = _log.warning
error = _log.error
debug = _log.debug
exception = _log.exception
fatal = _log.critical
INFO, WARNING, ERROR, DEBUG = _l.INFO, _l.WARNING, _l.ERROR, _l.DEBUG


def set_verbosity(v):
    _log.setLevel(v)


def get_absl_handler():
    return _l.StreamHandler()


class converter:  # noqa: N801  (absl.logging.converter, used by custom_logging.py:38)
    @staticmethod
    def get_initial_for_level(level):
        return _l.getLevelName(level)[:1]


# names custom_logging.py touches at import time (formatter/handler classes, level constants)
PythonFormatter = _l.Formatter
ABSLHandler = _l.StreamHandler
FATAL = _l.CRITICAL
_ABSL_LOG_FATAL = _l.CRITICAL
_CRITICAL_PREFIX = "F"
getLogger = _l.getLogger
