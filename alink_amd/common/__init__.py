"""Core data model: params, types, vectors, tables, mappers, model format, environment."""
