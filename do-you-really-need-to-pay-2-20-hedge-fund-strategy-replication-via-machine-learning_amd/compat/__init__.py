"""Reference-API compatibility layer (legacy class names, entry points, file naming)."""
