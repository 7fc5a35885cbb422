"""Drop-in mirrors of the reference's ``models`` package."""
