! Fortran 2008 bindings of the profiling API (reference
! parsec/fortran/parsec_profilef.F90): init / fini / reset / dump,
! dictionary keywords and user events.
module parsec_profile_f08
  use, intrinsic :: iso_c_binding
  implicit none

  interface
    subroutine parsec_profiling_init_c(basename, len, ierr) bind(C, name="parsec_profiling_init_f08")
      import :: c_char, c_int
      character(kind=c_char), dimension(*) :: basename
      integer(c_int), value :: len
      integer(c_int), intent(out) :: ierr
    end subroutine parsec_profiling_init_c
    function parsec_profiling_fini_f08() bind(C, name="parsec_profiling_fini") result(rc)
      import :: c_int
      integer(c_int) :: rc
    end function parsec_profiling_fini_f08
    function parsec_profiling_reset_f08() bind(C, name="parsec_profiling_reset") result(rc)
      import :: c_int
      integer(c_int) :: rc
    end function parsec_profiling_reset_f08
    function parsec_profiling_dbp_dump_f08() bind(C, name="parsec_profiling_dump") result(rc)
      import :: c_int
      integer(c_int) :: rc
    end function parsec_profiling_dbp_dump_f08
    subroutine parsec_profile_add_dictionary_keyword_c(name, name_len, attr, attr_len, info_len, key_start, key_end, ierr) &
        bind(C, name="parsec_profile_add_dictionary_keyword_f08")
      import :: c_char, c_int
      character(kind=c_char), dimension(*) :: name, attr
      integer(c_int), value :: name_len, attr_len, info_len
      integer(c_int), intent(out) :: key_start, key_end, ierr
    end subroutine parsec_profile_add_dictionary_keyword_c
    subroutine parsec_profiling_trace_f08(key, event_id, taskpool_id, ierr) bind(C, name="parsec_profiling_trace_f08")
      import :: c_int, c_int64_t
      integer(c_int), value :: key
      integer(c_int64_t), value :: event_id
      integer(c_int), value :: taskpool_id
      integer(c_int), intent(out) :: ierr
    end subroutine parsec_profiling_trace_f08
  end interface

contains

  subroutine parsec_profiling_init_f08(basename, ierr)
    character(len=*), intent(in) :: basename
    integer(c_int), intent(out) :: ierr
    call parsec_profiling_init_c(basename, int(len_trim(basename), c_int), ierr)
  end subroutine parsec_profiling_init_f08

  subroutine parsec_profile_add_dictionary_keyword_f08(name, attributes, info_length, key_start, key_end, ierr)
    character(len=*), intent(in) :: name, attributes
    integer(c_int), intent(in) :: info_length
    integer(c_int), intent(out) :: key_start, key_end, ierr
    call parsec_profile_add_dictionary_keyword_c(name, int(len_trim(name), c_int), attributes, int(len_trim(attributes), c_int), &
                                                 info_length, key_start, key_end, ierr)
  end subroutine parsec_profile_add_dictionary_keyword_f08

end module parsec_profile_f08
