import sys

from operator_amd.cli import main

sys.exit(main())
