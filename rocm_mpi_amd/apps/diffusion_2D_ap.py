"""Entry point mirroring scripts/diffusion_2D_ap.jl of the reference.

    python -m rocm_mpi_amd.apps.diffusion_2D_ap [--help]
    python -m rocm_mpi_amd.launch -n 4 -m rocm_mpi_amd.apps.diffusion_2D_ap
"""
import sys

from .cli import main_for

main = main_for("ap")

if __name__ == "__main__":
    sys.exit(main())
