"""Box ops, NMS wrapper, metrics."""
