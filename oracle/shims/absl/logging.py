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
