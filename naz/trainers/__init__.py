"""naz.trainers -> naz_amd.trainers."""
