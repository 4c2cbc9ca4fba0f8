"""Built-in game configurations (reference python/magent/builtin/config)."""
