import sys

from polyaxon_amd.cli.main import main

sys.exit(main())
