"""Drop-in mirror of the reference engine package (engine.engine.Engine)."""
