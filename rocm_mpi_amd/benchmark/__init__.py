"""Modules of the headline benchmark (``bench.py`` at the repository root is
the driver's entry point and keeps the CLI and the timed run): ``common``
(bounded collectives, failure protocol, watchdog), ``preflight``, ``checks``
(halo / drift / window / full-field), ``attribution`` (pass timings,
weak-scaling split)."""
