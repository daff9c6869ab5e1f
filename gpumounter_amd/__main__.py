import sys

from gpumounter_amd.cli import main

sys.exit(main())
