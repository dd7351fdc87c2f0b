__version__ = "1.4.1+mi355x_dp"
