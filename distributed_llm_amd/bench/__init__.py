"""bench"""
