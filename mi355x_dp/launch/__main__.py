import sys

from mi355x_dp.launch import main

sys.exit(main())
