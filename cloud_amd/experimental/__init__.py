"""Experimental APIs (reference ``TFC/experimental``)."""
