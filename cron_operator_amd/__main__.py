import sys

from .cmd.main import main

sys.exit(main())
