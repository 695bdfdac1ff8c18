"""Entry point mirroring scripts/diffusion_2D_perf_hide_prof.jl of the reference.

    python -m rocm_mpi_amd.apps.diffusion_2D_perf_hide_prof [--help]
    python -m rocm_mpi_amd.launch -n 4 -m rocm_mpi_amd.apps.diffusion_2D_perf_hide_prof
"""
import sys

from .cli import main_for

main = main_for("perf_hide_prof")

if __name__ == "__main__":
    sys.exit(main())
