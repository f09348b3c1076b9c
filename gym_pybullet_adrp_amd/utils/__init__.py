"""Host-side utilities: ABI mirror, enums, YAML race configs."""
