"""User-facing engine: YOLO model facade, inference sessions, results, validation."""
