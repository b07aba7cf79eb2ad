"""Empty torchaudio stand-in (only training-time criterion code touches it)."""
