"""Local stand-in for Amazon's ``smdistributed`` package, backed by mi355x_dp."""
