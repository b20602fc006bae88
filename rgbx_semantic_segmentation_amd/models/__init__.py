"""Drop-in mirror of the reference models package (models.builder.EncoderDecoder)."""
