"""torchtune stand-in: only modules.RotaryPositionalEmbeddings (restated)."""
