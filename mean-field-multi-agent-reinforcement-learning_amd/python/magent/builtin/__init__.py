"""Built-in configurations (reference python/magent/builtin)."""
