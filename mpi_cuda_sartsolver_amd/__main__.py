"""``python -m mpi_cuda_sartsolver_amd [options] input_files...`` -- the sartsolver CLI."""
import sys

from .cli import main

sys.exit(main())
