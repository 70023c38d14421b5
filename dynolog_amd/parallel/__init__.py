"""dynolog_amd.parallel"""
