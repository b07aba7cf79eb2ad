"""Shim (see ../__init__.py): the annotation target of custom_logging.py:226."""


class Fabric:  # noqa: D101
    pass
