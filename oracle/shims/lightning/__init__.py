"""Shim: lightning is absent here; the reference imports lightning.fabric only for a type
annotation (tts/utils/custom_logging.py:7,226).  No arithmetic."""
