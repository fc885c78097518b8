"""pools"""
