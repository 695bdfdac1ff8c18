"""Command-line entry points mirroring the reference scripts (scripts/*.jl)."""
