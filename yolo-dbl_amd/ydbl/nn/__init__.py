"""Model graph: YOLO-DBL modules (emit HIP launches) and YAML parsing."""
